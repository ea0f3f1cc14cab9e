#!/bin/bash
# The round's measurement evidence, in one GPU call (outputs under
# gpurun_out/, copy what is judged into profiles/<round>/ and profiles/pmc/):
#   bench_T_<tag>.txt            the default bench line (T)
#   prof_T_<tag>/ + .log         rocprofv3 --kernel-trace --stats of the same command
#   pmc/{T,C3,C5}_<tag>.json     PMC records keyed by kernel / build / workload
#   configs_<tag>.log            the single-GPU config lines
# Usage: scripts/round_evidence.sh <tag>
set -e
tag=$1
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench_T_$tag.txt 2>&1
scripts/prof_kernels.sh T_$tag --steps 3 --warmup 1 --no-cpu-baseline
bash scripts/pmc_workloads.sh $tag > gpurun_out/pmc_$tag.txt 2>&1
bash scripts/bench_configs.sh $tag > /dev/null
tail -1 gpurun_out/bench_T_$tag.txt | cut -c1-200
