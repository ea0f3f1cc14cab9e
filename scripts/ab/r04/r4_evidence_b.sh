#!/bin/bash
# round-4 evidence, part 2 (PMC records of part 1 committed under profiles/pmc/ first):
# fp32 PMC records, the default bench line, the config lines, fp32 lines, full C4 / C5
set -e
tag=$1
mkdir -p gpurun_out gpurun_out/pmc
scripts/pmc_passes.sh Tfp32_$tag --precision fp32 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmcf_$tag.txt 2>&1
scripts/pmc_passes.sh C2fp32_$tag --workload C2 --precision fp32 --steps 2 --warmup 1 --no-cpu-baseline >> gpurun_out/pmcf_$tag.txt 2>&1
scripts/pmc_passes.sh C3fp32_$tag --workload C3 --precision fp32 --steps 2 --warmup 1 --no-cpu-baseline >> gpurun_out/pmcf_$tag.txt 2>&1
cp gpurun_out/pmc/*fp32_$tag.json profiles/pmc/
timeout -k 10 300 python bench.py > gpurun_out/bench_T_$tag.txt 2>&1
tail -1 gpurun_out/bench_T_$tag.txt | cut -c1-300
bash scripts/bench_configs.sh $tag > /dev/null
bash scripts/bench_fp32.sh $tag > /dev/null
bash scripts/full_configs.sh $tag > /dev/null
