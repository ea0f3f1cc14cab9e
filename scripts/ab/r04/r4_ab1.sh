#!/bin/bash
# GPU suite, then interleaved A/B of the pinhole batch and one-quadratic media boundaries on C5 / C3 slices
set -e
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_r4b.txt 2>&1
tail -1 gpurun_out/gpu_tests_r4b.txt
B=raytracingweekend_amd/_build
bash scripts/ab_libs.sh r4b 3 "--workload C5 --spp 64" default $B/librtw_nopin.so $B/librtw_noquad.so $B/librtw_noboxrcp.so
bash scripts/ab_libs.sh r4b 3 "--workload C3 --spp 256" default $B/librtw_nopin.so
timeout -k 10 120 python bench.py --workload C5 --spp 64 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/c5_r4b.txt 2>&1
tail -1 gpurun_out/c5_r4b.txt | grep -o '"kernel": "[^"]*"\|"bvh_lds_nodes": [0-9]*'
