#!/bin/bash
# One GPU call's worth of checking: the GPU parity suite, the default bench
# line (T) and the single-GPU config lines, into gpurun_out/*_<tag>.*
# Usage: scripts/gpu_check.sh <tag> [--no-configs]
set -e
tag=$1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/gpu_tests_$tag.txt 2>&1
tail -3 gpurun_out/gpu_tests_$tag.txt
timeout -k 10 300 python bench.py > gpurun_out/bench_T_$tag.txt 2>&1
tail -1 gpurun_out/bench_T_$tag.txt
if [ "$2" != "--no-configs" ]; then
    bash scripts/bench_configs.sh $tag
fi
