#!/bin/bash
# round 5, call b: GPU suite (sqrt_core bit-exactness on the card, strict
# build, parity) on the tree with wave-uniform sqrt_core at the sqrt sites
# (RTW_SQRT_CORE, normalize included); A/B against librtw_sqbase (the
# compiler's sqrt everywhere), librtw_sqnonorm (normalize excluded) and
# librtw_nt (non-temporal radiance record stores)
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/gpu_tests_r5b.txt 2>&1
tail -n 1 gpurun_out/gpu_tests_r5b.txt
B=raytracingweekend_amd/_build
bash scripts/ab_libs.sh r5b_T 3 "--workload T" default $B/librtw_sqbase.so $B/librtw_sqnonorm.so $B/librtw_nt.so
bash scripts/ab_libs.sh r5b_C5 2 "--workload C5 --spp 64" default $B/librtw_sqbase.so $B/librtw_sqnonorm.so $B/librtw_nt.so
bash scripts/ab_libs.sh r5b_C3 2 "--workload C3 --spp 256" default $B/librtw_sqbase.so $B/librtw_sqnonorm.so
bash scripts/ab_libs.sh r5b_C2 2 "--workload C2" default $B/librtw_sqbase.so $B/librtw_sqnonorm.so
