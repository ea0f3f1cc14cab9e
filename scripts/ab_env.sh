#!/bin/bash
# A/B of environment settings over the BVH configs (short runs).
# Usage: scripts/ab_env.sh "VAR=a" "VAR=b" ...   ("-" = no setting)
mkdir -p gpurun_out
for cfg in "--scene random_balls --nx 1200 --ny 800 --spp 256 --bvh" \
           "--scene book2_final --nx 800 --ny 800 --spp 16 --bvh"; do
    for setting in "$@"; do
        if [ "$setting" = - ]; then envs=(); else envs=("$setting"); fi
        v=$(env "${envs[@]}" timeout -k 10 300 python bench.py $cfg --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-times | grep -o '"value": [0-9.]*')
        echo "$cfg | $setting | $v" | tee -a gpurun_out/ab_env.log
    done
done
