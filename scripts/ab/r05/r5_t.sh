#!/bin/bash
# round 5, call t: k_fast_sort's scene re-pointed with host-computed LDS
# offsets (RTW_FAST_LDS_OFF) -- fp32 bit-identity, A/B in-tree vs librtw_ldsoff0
set -e
B=raytracingweekend_amd/_build
mkdir -p gpurun_out
timeout -k 10 300 python scripts/lib_parity.py --fp32 $B/librtw_ldsoff0.so cornell_box light_sample random_balls | tee gpurun_out/parity_r5t.log
bash scripts/ab_libs.sh r5t_Tf 3 "--workload T --precision fp32" default $B/librtw_ldsoff0.so
bash scripts/ab_libs.sh r5t_T 2 "--workload T" default $B/librtw_ldsoff0.so
