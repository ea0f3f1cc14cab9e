#!/bin/bash
# 16-B BVH nodes (RTW_NODE16): GPU suite on the variant, then interleaved A/B on C5 slice, C3, C3 fp32
set -e
mkdir -p gpurun_out
B=raytracingweekend_amd/_build
RTW_LIBRARY=$B/librtw_node16.so timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_r4e_node16.txt 2>&1
tail -1 gpurun_out/gpu_tests_r4e_node16.txt
bash scripts/ab_libs.sh r4e 3 "--workload C5 --spp 64" default $B/librtw_node16.so
bash scripts/ab_libs.sh r4e 3 "--workload C3" default $B/librtw_node16.so
bash scripts/ab_libs.sh r4e 2 "--workload C3 --precision fp32" default $B/librtw_node16.so
