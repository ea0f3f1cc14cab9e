#!/bin/bash
# The BASELINE.json configs that fit one GPU, one bench line each, into
# gpurun_out/configs_<tag>.log: T, C2, C3 in full; C5 as a 64-spp slice of its
# 4096 (the full C5 / C4 are 8-GPU configs the driver runs).
# Usage: scripts/bench_configs.sh <tag> [extra bench args]
tag=$1; shift
out=gpurun_out/configs_$tag.log
mkdir -p gpurun_out; : > $out
run() { timeout -k 10 600 python bench.py --steps 2 --warmup 1 --no-cpu-baseline "$@" 2>/dev/null | tail -1 >> $out; }
run --workload T "$@"
run --workload C2 "$@"
run --workload C3 "$@"
run --workload C5 --spp 64 "$@"
run --scene book2_final --nx 800 --ny 800 --spp 16 "$@"                      # Book 2 flat list
python3 -c "
import json,sys
for l in open('$out'):
    d=json.loads(l); r=d.get('roofline') or {}
    print(d['config']['workload'], d['value'], d['unit'], r.get('kernel',''), 'lds_nodes', r.get('bvh_lds_nodes'))"
