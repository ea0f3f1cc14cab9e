#!/bin/bash
# radiance-only quotients as reciprocal products (radrcp) vs divisions (default): parity suite on the variant, T / C5 A/B
set -e
mkdir -p gpurun_out
B=raytracingweekend_amd/_build
RTW_LIBRARY=$B/librtw_radrcp.so timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_r4n_radrcp.txt 2>&1
tail -1 gpurun_out/gpu_tests_r4n_radrcp.txt
bash scripts/ab_libs.sh r4n 3 "--workload T" default $B/librtw_radrcp.so
bash scripts/ab_libs.sh r4n 2 "--workload C5 --spp 64" default $B/librtw_radrcp.so
