#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_bench_sizes.py -m gpu -x -v --timeout 300 --timeout-method thread -k whole > gpurun_out/gpu_tests_whole_r4w.txt 2>&1
tail -5 gpurun_out/gpu_tests_whole_r4w.txt
