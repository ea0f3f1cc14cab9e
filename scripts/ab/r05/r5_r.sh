#!/bin/bash
# round 5, call r: frames' second axis and lambertian normals normalised with
# the bare sqrt sequence (RTW_SQRT_UNIT) -- bit-identity, A/B in-tree vs librtw_unit0
set -e
B=raytracingweekend_amd/_build
mkdir -p gpurun_out
timeout -k 10 300 python scripts/lib_parity.py $B/librtw_unit0.so | tee gpurun_out/parity_r5r.log
bash scripts/ab_libs.sh r5r_T 3 "--workload T" default $B/librtw_unit0.so
bash scripts/ab_libs.sh r5r_C2 2 "--workload C2" default $B/librtw_unit0.so
bash scripts/ab_libs.sh r5r_C3 2 "--workload C3 --spp 256" default $B/librtw_unit0.so
bash scripts/ab_libs.sh r5r_C5 2 "--workload C5 --spp 64" default $B/librtw_unit0.so
