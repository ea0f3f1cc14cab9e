#!/bin/bash
# Interleaved A/B of environment settings on one workload (the in-tree library).
#   scripts/ab_env2.sh <tag> <rounds> "<bench args>" "ENV=val ..." "ENV=val ..." ...   ("-" = no setting)
set -e
tag=$1; rounds=$2; args=$3; shift 3
mkdir -p gpurun_out
for r in $(seq 1 "$rounds"); do
    for e in "$@"; do
        if [ "$e" = "-" ]; then envs=(); else read -r -a envs <<< "$e"; fi
        v=$(env "${envs[@]}" timeout -k 10 300 python bench.py $args --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-times | grep -o '"value": [0-9.]*')
        echo "round $r [$e] $args $v" | tee -a gpurun_out/ab_$tag.log
    done
done
