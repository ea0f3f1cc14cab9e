#!/bin/bash
# Section profile (lane-cycles per segment by phase, -DRTW_PROF library) of
# the persistent kernels on T, C3 and C5 slices -> gpurun_out/prof_<w>.txt
set -e
mkdir -p gpurun_out
export RTW_LIBRARY=raytracingweekend_amd/_build/librtw_prof.so
for w in "T --spp 128" "C3 --spp 128" "C5 --spp 16"; do
    n=${w%% *}
    timeout -k 10 200 python bench.py --workload $w --steps 1 --warmup 0 --no-cpu-baseline --no-kernel-times \
        > gpurun_out/prof_$n.txt 2>&1
    grep "rtw prof" gpurun_out/prof_$n.txt
done
