#!/bin/bash
# round 5, call q: the refill threshold re-measured on the final kernels
# (RTW_REFILL_MIN 8 in-tree vs 12 / 16): T, C2, T fp32 unaffected (k_fast_sort has none)
set -e
B=raytracingweekend_amd/_build
mkdir -p gpurun_out
bash scripts/ab_libs.sh r5q_T 3 "--workload T" default $B/librtw_rf12.so $B/librtw_rf16.so
bash scripts/ab_libs.sh r5q_C2 2 "--workload C2" default $B/librtw_rf12.so $B/librtw_rf16.so
