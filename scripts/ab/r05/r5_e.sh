#!/bin/bash
# round 5, call e: the fp32 Book-2 kernel in smaller workgroups --
# librtw_m896 (896 threads at 7 waves/SIMD, 9 spilled VGPRs, 1 632-node
# packet) and librtw_m768 (768 at 6 waves, spill-free, every node in the
# packet + its fetch shortcut) -- fp32 statistical parity tests on m768, then
# A/B against the in-tree build
set -e
mkdir -p gpurun_out
B=raytracingweekend_amd/_build
RTW_LIBRARY=$B/librtw_m768.so timeout -k 10 500 python -u -m pytest tests/test_gpu_fp32.py -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/gpu_tests_r5e_m768.txt 2>&1
tail -n 1 gpurun_out/gpu_tests_r5e_m768.txt
bash scripts/ab_libs.sh r5e_fmedia 3 "--workload C5 --spp 64 --precision fp32" default $B/librtw_m896.so $B/librtw_m768.so
