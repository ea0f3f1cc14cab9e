#!/bin/bash
# smoke() of the final build, and the fp32 C5 PMC record (k_fast for Book 2)
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r4v.txt 2>&1
tail -2 gpurun_out/smoke_r4v.txt
scripts/pmc_passes.sh C5fp32_r4v --workload C5 --spp 64 --precision fp32 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_c5f_r4v.txt 2>&1
tail -1 gpurun_out/pmc_c5f_r4v.txt | cut -c1-300
bash scripts/prof_sections.sh > gpurun_out/sections_r4v.txt 2>&1
cat gpurun_out/sections_r4v.txt
