#!/bin/bash
# round 5, call u: the world walk's rect test without its early return
# (RTW_RECT_BRANCHLESS) -- bit-identity, A/B librtw_rbl vs in-tree
set -e
B=raytracingweekend_amd/_build
mkdir -p gpurun_out
timeout -k 10 300 python scripts/lib_parity.py $B/librtw_rbl.so cornell_box light_sample random_balls | tee gpurun_out/parity_r5u.log
bash scripts/ab_libs.sh r5u_T 3 "--workload T" default $B/librtw_rbl.so
bash scripts/ab_libs.sh r5u_C5 2 "--workload C5 --spp 64" default $B/librtw_rbl.so
