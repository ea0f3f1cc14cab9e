#!/bin/bash
# GPU suite of the default build (medium cache and leaf reciprocals off), C5 A/B against
# the leaf-reciprocal variant, the C5 slice's sensitivity to the LDS node packet size,
# and PMC records of the fp32 fast mode (T, C3: spill write bytes vs records)
set -e
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_r4d.txt 2>&1
tail -1 gpurun_out/gpu_tests_r4d.txt
B=raytracingweekend_amd/_build
bash scripts/ab_libs.sh r4d 2 "--workload C5 --spp 64" default $B/librtw_leafrcp.so
for r in 1 2; do
  for n in - 768 384 0; do
    if [ $n = - ]; then envs=(); else envs=("RTW_LDS_NODES=$n"); fi
    v=$(env "${envs[@]}" timeout -k 10 300 python bench.py --workload C5 --spp 64 --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-times | grep -o '"value": [0-9.]*')
    echo "round $r C5 slice RTW_LDS_NODES=$n $v" | tee -a gpurun_out/ab_nodes_r4d.log
  done
done
scripts/pmc_passes.sh Tfp32_r4d --precision fp32 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_fp32_r4d.txt 2>&1
scripts/pmc_passes.sh C3fp32_r4d --workload C3 --precision fp32 --steps 2 --warmup 1 --no-cpu-baseline >> gpurun_out/pmc_fp32_r4d.txt 2>&1
tail -2 gpurun_out/pmc_fp32_r4d.txt | cut -c1-300
