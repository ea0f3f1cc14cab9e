#!/bin/bash
# round 5, call g: speculative group-BVH walks (RTW_SPEC_GROUP) now that the
# packet fetch is a plain LDS read: C5 / C3 slices, in-tree vs librtw_specg
set -e
B=raytracingweekend_amd/_build
bash scripts/ab_libs.sh r5g_specg 3 "--workload C5 --spp 64" default $B/librtw_specg.so
