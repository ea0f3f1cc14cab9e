#!/bin/bash
# Register / scratch / occupancy of ONE persistent-kernel instantiation,
# compiled alone (-DRTW_SUBSET: the launch tables keep just that one), for
# fast A/B of device-code changes on the CPU.
#   scripts/ru_kernel.sh F M LDS [extra hipcc flags...]   e.g.  scripts/ru_kernel.sh 112 8 true
# Writes /tmp/ru_<F>_<M>.txt (remarks) and /tmp/ks_<F>_<M>.s (ISA).
set -e
F=$1 M=$2 L=$3
shift 3
R=$(cd "$(dirname "$0")/.." && pwd)
B=$R/raytracingweekend_amd/csrc
FLAGS=(--offload-arch=gfx950 -munsafe-fp-atomics -fno-slp-vectorize -O3 -std=c++17 -fPIC -ffp-contract=off
       -fno-fast-math "-I$R/include" "-I$B" "-I$B/host" "-I$B/host/rtw" -DRTW_SUBSET -DRTW_SUBSET_F="$F"
       -DRTW_SUBSET_M="$M" -DRTW_SUBSET_L="$L" "$@" -x hip --offload-device-only)
/opt/rocm/bin/hipcc "${FLAGS[@]}" -c "$B/rtw_kernels.hip" -o /tmp/ru_$F_$M.o \
    -Rpass-analysis=kernel-resource-usage 2> "/tmp/ru_${F}_${M}.txt" || { tail -30 "/tmp/ru_${F}_${M}.txt"; exit 1; }
/opt/rocm/bin/hipcc "${FLAGS[@]}" -S "$B/rtw_kernels.hip" -o "/tmp/ks_${F}_${M}.s" 2>/dev/null
python3 "$R/scripts/resource_usage.py" "/tmp/ru_${F}_${M}.txt" k_persist
