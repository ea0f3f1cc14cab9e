#!/bin/bash
# d3 / double with one shared reciprocal (default) vs three divisions: GPU suite, then T / C2 / C3 / C5 A/B
set -e
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_r4m.txt 2>&1
tail -1 gpurun_out/gpu_tests_r4m.txt
B=raytracingweekend_amd/_build
bash scripts/ab_libs.sh r4m 3 "--workload T" default $B/librtw_nodiv3.so
bash scripts/ab_libs.sh r4m 2 "--workload C2" default $B/librtw_nodiv3.so
bash scripts/ab_libs.sh r4m 2 "--workload C3" default $B/librtw_nodiv3.so
bash scripts/ab_libs.sh r4m 2 "--workload C5 --spp 64" default $B/librtw_nodiv3.so
