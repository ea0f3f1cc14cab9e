#!/bin/bash
# round-4 evidence, part 1: GPU suite, rocprof stats of the default bench, fp64 PMC records
set -e
tag=$1
mkdir -p gpurun_out gpurun_out/pmc
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$tag.txt 2>&1
tail -1 gpurun_out/gpu_tests_$tag.txt
scripts/prof_kernels.sh T_$tag --steps 3 --warmup 1 --no-cpu-baseline
scripts/pmc_passes.sh T_$tag --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_$tag.txt 2>&1
scripts/pmc_passes.sh C2_$tag --workload C2 --steps 2 --warmup 1 --no-cpu-baseline >> gpurun_out/pmc_$tag.txt 2>&1
scripts/pmc_passes.sh C3_$tag --workload C3 --steps 2 --warmup 1 --no-cpu-baseline >> gpurun_out/pmc_$tag.txt 2>&1
scripts/pmc_passes.sh C5_$tag --workload C5 --spp 64 --steps 2 --warmup 1 --no-cpu-baseline >> gpurun_out/pmc_$tag.txt 2>&1
ls gpurun_out/pmc/
