#!/bin/bash
# Round-4 GPU check: VALU issue rates, the GPU suite, the default bench line,
# the config lines and the T PMC record of this build.
# Usage: scripts/r4_check.sh <tag> [--pmc T,C2,...] [--no-tests]
set -e
tag=$1; shift
pmc=""; tests=1
while [ $# -gt 0 ]; do
    case $1 in --pmc) pmc=$2; shift 2;; --no-tests) tests=0; shift;; *) shift;; esac
done
mkdir -p gpurun_out/pmc profiles/pmc
if [ -x scripts/bin/valu_rates ]; then timeout -k 10 60 scripts/bin/valu_rates > gpurun_out/valu_rates_$tag.log 2>&1; fi
if [ $tests = 1 ]; then
    timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
        > gpurun_out/gpu_tests_$tag.txt 2>&1
    tail -1 gpurun_out/gpu_tests_$tag.txt
fi
timeout -k 10 300 python bench.py > gpurun_out/bench_T_$tag.txt 2>&1
tail -1 gpurun_out/bench_T_$tag.txt | cut -c1-160
for w in ${pmc//,/ }; do
    case $w in
        C5) args="--workload C5 --spp 64";;
        *fp32) args="--workload ${w%fp32} --precision fp32";;
        *) args="--workload $w";;
    esac
    scripts/pmc_passes.sh ${w}_$tag $args --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_${w}_$tag.txt 2>&1
    cp gpurun_out/pmc/${w}_$tag.json profiles/pmc/
done
bash scripts/bench_configs.sh $tag
