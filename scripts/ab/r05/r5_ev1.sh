#!/bin/bash
# round 5 evidence, part 1 (tag $1): GPU suite, rocprof of the default bench
# command, PMC records of the fp64 workloads T, C2, C3, C5 (64-spp slice)
set -e
tag=$1
mkdir -p gpurun_out profiles/pmc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/gpu_tests_$tag.txt 2>&1
tail -n 1 gpurun_out/gpu_tests_$tag.txt
scripts/prof_kernels.sh T_$tag --steps 3 --warmup 1 --no-cpu-baseline
for w in "T_$tag" "C2_$tag --workload C2" "C3_$tag --workload C3" "C5_$tag --workload C5 --spp 64"; do
    set -- $w
    t=$1; shift
    scripts/pmc_passes.sh $t "$@" --steps 2 --warmup 1 --no-cpu-baseline
    echo "pmc $t done"
done
ls gpurun_out/pmc/
