#!/bin/bash
# round 5, call d: GPU parity tests on librtw_tos (top-of-stack register in
# the group / fp32 world walks, fp32 all-in-packet fetch outside the media
# kernel), then A/B against the in-tree build
set -e
mkdir -p gpurun_out
B=raytracingweekend_amd/_build
RTW_LIBRARY=$B/librtw_tos.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_sizes.py tests/test_gpu_fp32.py -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/gpu_tests_r5d_tos.txt 2>&1
tail -n 1 gpurun_out/gpu_tests_r5d_tos.txt
bash scripts/ab_libs.sh r5d_C5 3 "--workload C5 --spp 64" default $B/librtw_tos.so
bash scripts/ab_libs.sh r5d_C3 2 "--workload C3 --spp 256" default $B/librtw_tos.so
bash scripts/ab_libs.sh r5d_T 2 "--workload T" default $B/librtw_tos.so
bash scripts/ab_libs.sh r5d_f32 2 "--workload C3 --precision fp32" default $B/librtw_tos.so
bash scripts/ab_libs.sh r5d_f32 2 "--workload C5 --spp 64 --precision fp32" default $B/librtw_tos.so
