#!/bin/bash
# The two 8-GPU configs (C4 Cornell 800x800x4096, C5 Book-2 final
# 1600x1600x4096) rendered at full size on ONE GPU -- the N = 1 points of the
# strong-scaling curve -- one bench line each into gpurun_out/full_<tag>.log,
# plus rocprof kernel stats of the same commands.
# Usage: scripts/full_configs.sh <tag> [extra bench args]
set -e
tag=$1; shift
out=gpurun_out/full_$tag.log
mkdir -p gpurun_out; : > $out
run() {
    timeout -k 10 400 python bench.py --steps 1 --warmup 1 "$@" > gpurun_out/full_$tag.tmp 2>&1 \
        || { cat gpurun_out/full_$tag.tmp; exit 1; }
    tail -1 gpurun_out/full_$tag.tmp >> $out
    tail -1 gpurun_out/full_$tag.tmp | cut -c1-400
}
run --workload C4 "$@"
run --workload C5 "$@"
rm -f gpurun_out/full_$tag.tmp
