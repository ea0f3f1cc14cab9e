#!/bin/bash
# Interleaved A/B of library variants on one workload.
#   scripts/ab_libs.sh <tag> <rounds> "<bench args>" lib1 lib2 ...   ("default" = in-tree librtw.so)
set -e
tag=$1; rounds=$2; args=$3; shift 3
mkdir -p gpurun_out
for r in $(seq 1 "$rounds"); do
    for lib in "$@"; do
        if [ "$lib" = default ]; then unset RTW_LIBRARY; else export RTW_LIBRARY=$lib; fi
        v=$(timeout -k 10 300 python bench.py $args --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-times | grep -o '"value": [0-9.]*')
        echo "round $r $lib $args $v" | tee -a gpurun_out/ab_$tag.log
    done
done
