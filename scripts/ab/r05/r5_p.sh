#!/bin/bash
# round 5, call p: pinhole directions normalised with one shared reciprocal
# where the host proved the ranges (RTW_CAM_DIR_RCP) -- bit-identity, A/B
# in-tree vs librtw_camold
set -e
B=raytracingweekend_amd/_build
mkdir -p gpurun_out
timeout -k 10 300 python scripts/lib_parity.py $B/librtw_camold.so | tee gpurun_out/parity_r5p.log
bash scripts/ab_libs.sh r5p_T 3 "--workload T" default $B/librtw_camold.so
bash scripts/ab_libs.sh r5p_C2 2 "--workload C2" default $B/librtw_camold.so
bash scripts/ab_libs.sh r5p_C3 2 "--workload C3 --spp 256" default $B/librtw_camold.so
bash scripts/ab_libs.sh r5p_C5 2 "--workload C5 --spp 64" default $B/librtw_camold.so
