#!/bin/bash
# AMDGPU machine-scheduler strategies (whole library): default vs max-ilp vs max-memory-clause on T, C2, C3, C5
set -e
mkdir -p gpurun_out
B=raytracingweekend_amd/_build
bash scripts/ab_libs.sh r4s 3 "--workload T" default $B/librtw_maxilp.so $B/librtw_memclause.so
bash scripts/ab_libs.sh r4s 2 "--workload C2" default $B/librtw_maxilp.so $B/librtw_memclause.so
bash scripts/ab_libs.sh r4s 2 "--workload C3" default $B/librtw_maxilp.so $B/librtw_memclause.so
bash scripts/ab_libs.sh r4s 2 "--workload C5 --spp 64" default $B/librtw_maxilp.so $B/librtw_memclause.so
