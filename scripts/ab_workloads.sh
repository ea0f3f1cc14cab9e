#!/bin/bash
# Interleaved A/B of library variants over the single-GPU workloads (T, C2,
# a C3 slice, a C5 slice).
#   scripts/ab_workloads.sh <tag> <rounds> lib1 lib2 ...   ("default" = in-tree librtw.so)
set -e
tag=$1; rounds=$2; shift 2
for w in "--workload T" "--workload C2" "--workload C3 --spp 256" "--workload C5 --spp 64"; do
    bash "$(dirname "$0")/ab_libs.sh" "$tag" "$rounds" "$w" "$@"
done
