#!/bin/bash
# The BASELINE.json configs that fit one GPU, one bench line each, into
# gpurun_out/configs_<tag>.log.  Usage: scripts/bench_configs.sh <tag> [extra bench args]
tag=$1; shift
out=gpurun_out/configs_$tag.log
mkdir -p gpurun_out; : > $out
run() { timeout -k 10 600 python bench.py --steps 2 --warmup 1 --no-cpu-baseline "$@" 2>/dev/null | tail -1 >> $out; }
run --scene cornell_box --nx 800 --ny 800 --spp 1024 "$@"                    # T
run --scene random_balls --nx 1200 --ny 800 --spp 256 "$@"                   # C2 flat
run --scene random_balls --nx 1200 --ny 800 --spp 1024 --bvh "$@"            # C3 BVH
run --scene book2_final --nx 1600 --ny 1600 --spp 64 --bvh "$@"              # C5 (per-GPU slice: 64 of 4096 spp)
run --scene book2_final --nx 800 --ny 800 --spp 16 "$@"                      # Book 2 flat list
cat $out | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['config']['workload'], d['value'], d['unit'], d['roofline']['kernel'] if d.get('roofline') else '')"
