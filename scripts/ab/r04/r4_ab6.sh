#!/bin/bash
# fp32-reciprocal slab rays (default now) vs fp64 divisions; BVH kernels at 768 threads / 3 waves (no spills)
set -e
mkdir -p gpurun_out
timeout -k 10 120 python -u -m pytest tests/test_slab32.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_r4h_quick.txt 2>&1
tail -1 gpurun_out/gpu_tests_r4h_quick.txt
B=raytracingweekend_amd/_build
bash scripts/ab_libs.sh r4h 3 "--workload C5 --spp 64" default $B/librtw_slabdiv.so $B/librtw_b768w3.so
bash scripts/ab_libs.sh r4h 2 "--workload C3" default $B/librtw_slabdiv.so $B/librtw_b768w3.so
