#!/bin/bash
set -e
B=raytracingweekend_amd/_build
mkdir -p gpurun_out
timeout -k 10 300 python scripts/lib_parity.py $B/librtw_lpbl.so cornell_box light_sample | tee gpurun_out/parity_r5w.log
bash scripts/ab_libs.sh r5w_T 3 "--workload T" default $B/librtw_lpbl.so
