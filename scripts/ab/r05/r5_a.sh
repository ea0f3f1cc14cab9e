#!/bin/bash
# round 5, call a: GPU suite on the tree, then fp32 Book-2 kernel with its
# throughput / sample id in LDS home slots (librtw_fhome) vs the in-tree one,
# and the home variant's HBM write bytes (one PMC pass)
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_r5a.txt 2>&1
tail -n 1 gpurun_out/gpu_tests_r5a.txt
B=raytracingweekend_amd/_build
bash scripts/ab_libs.sh r5a 3 "--workload C5 --spp 64 --precision fp32" default $B/librtw_fhome.so
export RTW_LIBRARY=$B/librtw_fhome.so
bash scripts/prof_pmc.sh C5fp32home_w "WRITE_SIZE GRBM_COUNT" --workload C5 --spp 64 --precision fp32 --steps 2 --warmup 1 --no-cpu-baseline
unset RTW_LIBRARY
bash scripts/prof_pmc.sh C5fp32_w "WRITE_SIZE GRBM_COUNT" --workload C5 --spp 64 --precision fp32 --steps 2 --warmup 1 --no-cpu-baseline
