#!/bin/bash
# The round's measurement evidence, in one GPU call (outputs under
# gpurun_out/, copy what is judged into profiles/<round>/ and profiles/pmc/):
#   gpu_tests_<tag>.txt          the GPU parity suite
#   prof_T_<tag>/ + .log         rocprofv3 --kernel-trace --stats of the default bench command
#   pmc/{T,C3,C5}_<tag>.json     PMC records keyed by kernel / build / workload
#   bench_T_<tag>.txt            the default bench line (T), run after the PMC
#                                records are in profiles/pmc/ so its roofline
#                                carries the record of this very build
#   configs_<tag>.log            the single-GPU config lines (same)
# Usage: scripts/round_evidence.sh <tag> [--no-tests]
set -e
tag=$1
mkdir -p gpurun_out profiles/pmc
if [ "$2" != "--no-tests" ]; then
    timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
        > gpurun_out/gpu_tests_$tag.txt 2>&1
    tail -1 gpurun_out/gpu_tests_$tag.txt
fi
scripts/prof_kernels.sh T_$tag --steps 3 --warmup 1 --no-cpu-baseline
bash scripts/pmc_workloads.sh $tag > gpurun_out/pmc_$tag.txt 2>&1
cp gpurun_out/pmc/*_$tag.json profiles/pmc/
timeout -k 10 300 python bench.py > gpurun_out/bench_T_$tag.txt 2>&1
tail -1 gpurun_out/bench_T_$tag.txt | cut -c1-200
bash scripts/bench_configs.sh $tag > /dev/null
bash scripts/bench_fp32.sh $tag > /dev/null
bash scripts/full_configs.sh $tag > /dev/null
