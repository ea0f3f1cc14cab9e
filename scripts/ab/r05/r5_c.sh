#!/bin/bash
# round 5, call c: parity of librtw_both (two-step RNG jumps in the rejection
# loops + the all-in-packet node fetch) on the GPU parity tests, then A/B of
# the in-tree build against librtw_jump / librtw_pall / librtw_both
set -e
mkdir -p gpurun_out
B=raytracingweekend_amd/_build
RTW_LIBRARY=$B/librtw_both.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_sizes.py -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/gpu_tests_r5c_both.txt 2>&1
tail -n 1 gpurun_out/gpu_tests_r5c_both.txt
bash scripts/ab_libs.sh r5c_T 3 "--workload T" default $B/librtw_jump.so $B/librtw_pall.so $B/librtw_both.so
bash scripts/ab_libs.sh r5c_C5 2 "--workload C5 --spp 64" default $B/librtw_jump.so $B/librtw_pall.so $B/librtw_both.so
bash scripts/ab_libs.sh r5c_C2 2 "--workload C2" default $B/librtw_jump.so $B/librtw_both.so
bash scripts/ab_libs.sh r5c_C3 2 "--workload C3 --spp 256" default $B/librtw_jump.so $B/librtw_both.so
