#!/bin/bash
# GPU suite on the working tree, then interleaved A/B of the in-tree library
# against _build/librtw_base.so (HEAD kernels) on T, a C5 slice and a C3 slice.
#   scripts/ab_quick.sh <tag> <rounds> [--no-tests]
set -e
tag=$1; rounds=$2
mkdir -p gpurun_out
if [ "$3" != "--no-tests" ]; then
    timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
        > gpurun_out/gpu_tests_$tag.txt 2>&1 || { tail -30 gpurun_out/gpu_tests_$tag.txt; exit 1; }
    tail -2 gpurun_out/gpu_tests_$tag.txt
fi
for r in $(seq 1 "$rounds"); do
    for lib in default raytracingweekend_amd/_build/librtw_base.so; do
        for w in "--workload T" "--workload C5 --spp 64" "--workload C3 --spp 256"; do
            if [ "$lib" = default ]; then unset RTW_LIBRARY; else export RTW_LIBRARY=$lib; fi
            v=$(timeout -k 10 300 python bench.py $w --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-times | grep -o '"value": [0-9.]*')
            echo "round $r $lib $w $v" | tee -a gpurun_out/ab_$tag.log
        done
    done
done
