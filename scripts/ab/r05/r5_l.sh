#!/bin/bash
# round 5, call l: the counting sort's block prefix by DPP (RTW_SORT_DPP) --
# bit-identity fp64 / fp32, then T, C2, T fp32, C2 fp32: in-tree vs librtw_dpp
set -e
B=raytracingweekend_amd/_build
mkdir -p gpurun_out
timeout -k 10 300 python scripts/lib_parity.py $B/librtw_dpp.so cornell_box random_balls light_sample | tee gpurun_out/parity_r5l.log
timeout -k 10 300 python scripts/lib_parity.py --fp32 $B/librtw_dpp.so cornell_box random_balls | tee -a gpurun_out/parity_r5l.log
bash scripts/ab_libs.sh r5l_T 3 "--workload T" default $B/librtw_dpp.so
bash scripts/ab_libs.sh r5l_C2 2 "--workload C2" default $B/librtw_dpp.so
bash scripts/ab_libs.sh r5l_Tf 2 "--workload T --precision fp32" default $B/librtw_dpp.so
bash scripts/ab_libs.sh r5l_C2f 2 "--workload C2 --precision fp32" default $B/librtw_dpp.so
