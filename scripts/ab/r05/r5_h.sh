#!/bin/bash
# round 5, call h: mixture choice sorted on (RTW_SORT_MIXTURE) -- bit-identity
# on four scenes, then T A/B, in-tree vs librtw_mix
set -e
B=raytracingweekend_amd/_build
mkdir -p gpurun_out
timeout -k 10 400 python scripts/lib_parity.py $B/librtw_mix.so | tee gpurun_out/parity_r5h.log
bash scripts/ab_libs.sh r5h_mix 3 "--workload T" default $B/librtw_mix.so
