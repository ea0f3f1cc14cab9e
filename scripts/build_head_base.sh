#!/bin/bash
# Build _build/librtw_base.so from the committed HEAD kernels (A/B baseline
# for uncommitted kernel changes; host objects from the in-tree build).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
git -C "$R" archive HEAD raytracingweekend_amd/csrc | tar -x -C "$T"
"$R/scripts/build_alt.sh" "$T/raytracingweekend_amd/csrc" base
rm -rf "$T"
