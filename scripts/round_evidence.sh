#!/bin/bash
# The round's measurement evidence for the T workload, in one GPU call:
# the default bench line, rocprofv3 kernel stats of the same command, the
# PMC passes (scripts/pmc_passes.sh) and the single-GPU config lines.
# Usage: scripts/round_evidence.sh <tag>   (outputs under gpurun_out/)
set -e
tag=$1
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench_T_$tag.log 2>&1
scripts/prof_kernels.sh T_$tag --steps 3 --warmup 1 --no-cpu-baseline
scripts/pmc_passes.sh T_$tag --steps 2 --warmup 1 --no-cpu-baseline
bash scripts/bench_configs.sh $tag > /dev/null
