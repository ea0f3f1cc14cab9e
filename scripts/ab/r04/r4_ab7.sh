#!/bin/bash
# fused group-BVH walks (default) vs separate walks: GPU suite (parity), then C5 slice / C3 A/B
set -e
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_r4j.txt 2>&1
tail -1 gpurun_out/gpu_tests_r4j.txt
B=raytracingweekend_amd/_build
bash scripts/ab_libs.sh r4j 3 "--workload C5 --spp 64" default $B/librtw_nofuse.so
