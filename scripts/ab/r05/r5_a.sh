#!/bin/bash
# round 5, call a: GPU suite on the tree; T: in-tree (one-step canonical
# division) vs librtw_canon2 (two steps) vs librtw_hr (home-slot rays in
# k_persist_sort); fp32 Book-2 kernel with throughput / sample id in LDS
# home slots (librtw_fhome) vs in-tree, and both kernels' HBM write bytes;
# fp64 Book-2 kernel with the ray parked in LDS and lane-direct camera
# samples (librtw_direct) vs in-tree
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/gpu_tests_r5a.txt 2>&1
tail -n 1 gpurun_out/gpu_tests_r5a.txt
B=raytracingweekend_amd/_build
bash scripts/ab_libs.sh r5a_T 3 "--workload T" default $B/librtw_canon2.so $B/librtw_hr.so
bash scripts/ab_libs.sh r5a_C5 3 "--workload C5 --spp 64" default $B/librtw_direct.so
bash scripts/ab_libs.sh r5a_C5f 3 "--workload C5 --spp 64 --precision fp32" default $B/librtw_fhome.so
export RTW_LIBRARY=$B/librtw_fhome.so
bash scripts/prof_pmc.sh C5fp32home_w "WRITE_SIZE GRBM_COUNT" --workload C5 --spp 64 --precision fp32 --steps 2 --warmup 1 --no-cpu-baseline
unset RTW_LIBRARY
bash scripts/prof_pmc.sh C5fp32_w "WRITE_SIZE GRBM_COUNT" --workload C5 --spp 64 --precision fp32 --steps 2 --warmup 1 --no-cpu-baseline
