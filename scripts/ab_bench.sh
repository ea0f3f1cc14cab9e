#!/bin/bash
# A/B of library variants on one box: interleaved rounds of a short bench
# per variant.  Usage: scripts/ab_bench.sh <rounds> "<bench args>" lib1 lib2 ...
# (lib = path of a librtw*.so; "default" = the in-tree librtw.so)
set -e
rounds=$1; shift
args=$1; shift
mkdir -p gpurun_out
for r in $(seq 1 "$rounds"); do
    for lib in "$@"; do
        if [ "$lib" = default ]; then unset RTW_LIBRARY; else export RTW_LIBRARY=$lib; fi
        v=$(timeout -k 10 300 python bench.py $args --no-cpu-baseline --no-kernel-times | grep -o '"value": [0-9.]*')
        echo "round $r $lib $v" | tee -a gpurun_out/ab.log
    done
done
