#!/bin/bash
# A/B of environment settings over the BVH workloads C3 and a C5 slice
# (interleaved, short runs) into gpurun_out/ab_env.log.
# Usage: scripts/ab_env.sh <rounds> "VAR=a" "VAR=b" ...   ("-" = no setting)
mkdir -p gpurun_out
rounds=$1; shift
for r in $(seq 1 "$rounds"); do
    for cfg in "--workload C3" "--workload C5 --spp 64"; do
        for setting in "$@"; do
            if [ "$setting" = - ]; then envs=(); else envs=("$setting"); fi
            v=$(env "${envs[@]}" timeout -k 10 300 python bench.py $cfg --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-times | grep -o '"value": [0-9.]*')
            echo "round $r | $cfg | $setting | $v" | tee -a gpurun_out/ab_env.log
        done
    done
done
