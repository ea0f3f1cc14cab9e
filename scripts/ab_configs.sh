#!/bin/bash
# A/B of library variants over the single-GPU BASELINE configs (short runs).
# Usage: scripts/ab_configs.sh lib1 lib2 ...   ("default" = in-tree librtw.so)
mkdir -p gpurun_out
for cfg in "--scene cornell_box --nx 800 --ny 800 --spp 256" \
           "--scene random_balls --nx 1200 --ny 800 --spp 64" \
           "--scene random_balls --nx 1200 --ny 800 --spp 256 --bvh" \
           "--scene book2_final --nx 800 --ny 800 --spp 16 --bvh" \
           "--scene book2_final --nx 400 --ny 400 --spp 8"; do
    for lib in "$@"; do
        if [ "$lib" = default ]; then unset RTW_LIBRARY; else export RTW_LIBRARY=$lib; fi
        v=$(timeout -k 10 300 python bench.py $cfg --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-times | grep -o '"value": [0-9.]*')
        echo "$cfg | $lib | $v" | tee -a gpurun_out/ab_configs.log
    done
done
