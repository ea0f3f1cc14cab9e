#!/bin/bash
# Build a variant librtw from an alternative kernel source tree (tuning A/B):
#   [EXTRA="<hipcc flags>"] scripts/build_alt.sh <csrc-dir> <name>  ->  raytracingweekend_amd/_build/librtw_<name>.so
# Host objects come from the in-tree build (run the normal build first).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
D=$1; N=$2
B=$R/raytracingweekend_amd/_build
/opt/rocm/bin/hipcc --offload-arch=gfx950 -munsafe-fp-atomics -fno-slp-vectorize -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math $EXTRA \
    -I$R/include -I$D -I$D/host -I$D/host/rtw -x hip -c $D/rtw_kernels.hip -o $B/alt_$N.o
host=$(ls $B/*.cpp.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $B/alt_$N.o $host -o $B/librtw_$N.so
echo $B/librtw_$N.so
