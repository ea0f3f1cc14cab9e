#!/bin/bash
# rejection loops (unit sphere, camera disk) decided in fp32 (default) vs fp64 (norej): GPU suite, then A/B
set -e
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_r4t.txt 2>&1
tail -1 gpurun_out/gpu_tests_r4t.txt
B=raytracingweekend_amd/_build
bash scripts/ab_libs.sh r4t 3 "--workload C5 --spp 64" default $B/librtw_norej.so
bash scripts/ab_libs.sh r4t 2 "--workload C3" default $B/librtw_norej.so
bash scripts/ab_libs.sh r4t 2 "--workload C2" default $B/librtw_norej.so
bash scripts/ab_libs.sh r4t 3 "--workload T" default $B/librtw_norej.so
