#!/bin/bash
# fused group-BVH walks, one walk site (fuse3) vs separate walks (default): parity suite on the variant, C5 A/B
set -e
mkdir -p gpurun_out
B=raytracingweekend_amd/_build
RTW_LIBRARY=$B/librtw_fuse3.so timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_r4k_fuse3.txt 2>&1
tail -1 gpurun_out/gpu_tests_r4k_fuse3.txt
bash scripts/ab_libs.sh r4k 3 "--workload C5 --spp 64" default $B/librtw_fuse3.so
