#!/bin/bash
# round 5, call v: the branchless world rects' winner taken with selects
# (RTW_RECT_SELECT) -- bit-identity, A/B in-tree vs librtw_sel0
set -e
B=raytracingweekend_amd/_build
mkdir -p gpurun_out
timeout -k 10 300 python scripts/lib_parity.py $B/librtw_sel0.so cornell_box light_sample random_balls | tee gpurun_out/parity_r5v.log
bash scripts/ab_libs.sh r5v_T 3 "--workload T" default $B/librtw_sel0.so
bash scripts/ab_libs.sh r5v_C5 2 "--workload C5 --spp 64" default $B/librtw_sel0.so
