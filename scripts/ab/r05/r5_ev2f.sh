#!/bin/bash
# round 5 evidence part 2 for build tag $1 (scripts/ab/r05/r5_ev2.sh), then
# A/B: the all-in-packet node fetch in the fp32 walks (librtw_fpall) vs in-tree
set -e
tag=$1
bash scripts/ab/r05/r5_ev2.sh $tag
B=raytracingweekend_amd/_build
bash scripts/ab_libs.sh r5f_fpall 2 "--workload C3 --precision fp32" default $B/librtw_fpall.so
bash scripts/ab_libs.sh r5f_fpall 2 "--workload T --precision fp32" default $B/librtw_fpall.so
bash scripts/ab_libs.sh r5f_fpall 2 "--workload C5 --spp 64 --precision fp32" default $B/librtw_fpall.so
