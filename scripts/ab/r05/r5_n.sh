#!/bin/bash
# round 5, call n: libstdc++'s canonical clamp as one v_min_f64 (RTW_CANON_MIN)
# -- bit-identity, then A/B in-tree vs librtw_nomin
set -e
B=raytracingweekend_amd/_build
mkdir -p gpurun_out
timeout -k 10 300 python scripts/lib_parity.py $B/librtw_nomin.so | tee gpurun_out/parity_r5n.log
bash scripts/ab_libs.sh r5n_T 3 "--workload T" default $B/librtw_nomin.so
bash scripts/ab_libs.sh r5n_C3 2 "--workload C3 --spp 256" default $B/librtw_nomin.so
bash scripts/ab_libs.sh r5n_C5 2 "--workload C5 --spp 64" default $B/librtw_nomin.so
bash scripts/ab_libs.sh r5n_C2 2 "--workload C2" default $B/librtw_nomin.so
