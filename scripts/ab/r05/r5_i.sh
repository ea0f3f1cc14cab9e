#!/bin/bash
# round 5, call i: 16-byte BVH nodes for the fp32 media kernel (every C5 node
# in the LDS packet), with and without the all-in-packet fetch: fp32
# bit-identity, then C5 fp32 slices, in-tree vs librtw_n16 / librtw_n16p
set -e
B=raytracingweekend_amd/_build
mkdir -p gpurun_out
for v in n16 n16p; do
    timeout -k 10 300 python scripts/lib_parity.py --fp32 $B/librtw_$v.so book2_final random_balls | tee -a gpurun_out/parity_r5i.log
done
bash scripts/ab_libs.sh r5i_n16 3 "--workload C5 --spp 64 --precision fp32" default $B/librtw_n16.so $B/librtw_n16p.so
