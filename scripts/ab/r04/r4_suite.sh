#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_final_r4x.txt 2>&1
tail -2 gpurun_out/gpu_tests_final_r4x.txt
