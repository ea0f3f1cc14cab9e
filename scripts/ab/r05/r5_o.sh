#!/bin/bash
# round 5, call o: the per-sample seed's remainder folded in 32-bit steps
# (RTW_SEED_FOLD) -- bit-identity, then A/B in-tree vs librtw_seedold
set -e
B=raytracingweekend_amd/_build
mkdir -p gpurun_out
timeout -k 10 300 python scripts/lib_parity.py $B/librtw_seedold.so | tee gpurun_out/parity_r5o.log
timeout -k 10 300 python scripts/lib_parity.py --fp32 $B/librtw_seedold.so cornell_box | tee -a gpurun_out/parity_r5o.log
bash scripts/ab_libs.sh r5o_T 4 "--workload T" default $B/librtw_seedold.so
bash scripts/ab_libs.sh r5o_C3 2 "--workload C3 --spp 256" default $B/librtw_seedold.so
bash scripts/ab_libs.sh r5o_Tf 2 "--workload T --precision fp32" default $B/librtw_seedold.so
