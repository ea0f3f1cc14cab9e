#!/bin/bash
# fp32 fast-mode bench lines (statistical parity; never the headline) for the
# single-GPU workloads: T, C2, C3, C4, C5 -> gpurun_out/fp32_<tag>.log
# Usage: scripts/bench_fp32.sh <tag>
tag=$1
out=gpurun_out/fp32_$tag.log
mkdir -p gpurun_out; : > $out
run() { timeout -k 10 600 python bench.py --precision fp32 --steps 2 --warmup 1 --no-cpu-baseline "$@" 2>/dev/null | tail -1 >> $out; }
run --workload T
run --workload C2
run --workload C3
run --workload C4 --steps 1
run --workload C5 --steps 1
python3 -c "
import json
for l in open('$out'):
    d=json.loads(l); r=d.get('roofline') or {}
    print(d['config']['workload'], d['dtype'], d['value'], d['unit'], r.get('kernel',''), d.get('segments_per_sample'))"
