#!/bin/bash
# round 5, call j: the N > 1 bench path rehearsed on one GPU (RTW_BENCH_SHARED_GPU=1:
# every rank on cuda:0, gloo collectives) at the full T workload, N = 1, 2, 4
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_multirank.py -x -v -s --timeout 200 --timeout-method thread \
    > gpurun_out/multirank_r5j.txt 2>&1
for n in 1 2 4; do
    RTW_BENCH_SHARED_GPU=1 timeout -k 10 300 python bench.py --gpus $n --steps 3 --warmup 1 --no-cpu-baseline \
        > gpurun_out/rehearsal_T_n$n.txt 2>&1
    grep '^{' gpurun_out/rehearsal_T_n$n.txt
done
