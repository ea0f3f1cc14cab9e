#!/bin/bash
# GPU suite, then interleaved A/B: media boundary cache and per-leaf reciprocals (C5 slice), refill threshold (T, C2)
set -e
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_r4c.txt 2>&1
tail -1 gpurun_out/gpu_tests_r4c.txt
B=raytracingweekend_amd/_build
bash scripts/ab_libs.sh r4c 3 "--workload C5 --spp 64" default $B/librtw_nocache.so $B/librtw_noleafrcp.so
bash scripts/ab_libs.sh r4c 3 "--workload T" default $B/librtw_refill16.so $B/librtw_refill4.so
bash scripts/ab_libs.sh r4c 2 "--workload C2" default $B/librtw_refill16.so $B/librtw_refill4.so
for w in T C2 C3; do
  timeout -k 10 300 python bench.py --precision fp32 --workload $w --steps 2 --warmup 1 --no-cpu-baseline >> gpurun_out/fp32_r4c.log 2>&1
done
tail -3 gpurun_out/fp32_r4c.log
