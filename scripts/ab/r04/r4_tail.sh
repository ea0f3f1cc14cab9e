#!/bin/bash
# where the fixed per-step time goes at the 8-GPU share of T (128 spp): kernel trace of a short bench
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/prof_T128_r4r -o run --output-format csv -- \
    python3 bench.py --workload T --spp 128 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_T128_r4r.log 2>&1
tail -1 gpurun_out/prof_T128_r4r.log | cut -c1-200
