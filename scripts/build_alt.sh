#!/bin/bash
# Build a variant librtw from an alternative kernel source tree (tuning A/B):
#   [EXTRA="<hipcc flags>"] scripts/build_alt.sh <csrc-dir> <name>  ->  raytracingweekend_amd/_build/librtw_<name>.so
# The host objects are brought up to date first (the in-tree build), so the
# variant links the current host library.  EXTRA is split on whitespace on
# purpose (several flags in one variable).
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
D=$1
N=$2
B="$R/raytracingweekend_amd/_build"
(cd "$R" && python3 -c "from raytracingweekend_amd import build; build.build_library()")
read -r -a extra <<< "${EXTRA:-}"
bid=$(cd "$R" && python3 -c "from raytracingweekend_amd import build; print(build.build_id(['alt:$N'] + '${EXTRA:-}'.split()))")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -munsafe-fp-atomics -fno-slp-vectorize -O3 -std=c++17 -fPIC \
    -ffp-contract=off -fno-fast-math "${extra[@]}" "-DRTW_BUILD_ID=\"$bid\"" \
    -I"$R/include" -I"$D" -I"$D/host" -I"$D/host/rtw" -x hip -c "$D/rtw_kernels.hip" -o "$B/alt_$N.o"
host=("$B"/*.cpp.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC "$B/alt_$N.o" "${host[@]}" -L/opt/rocm/lib -lrccl \
    -o "$B/librtw_$N.so"
echo "$B/librtw_$N.so"
