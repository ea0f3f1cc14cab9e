#!/bin/bash
# round 5, call k: overlapped passes (RTW_OVERLAP=n) -- bit-identity on five
# cases, then env A/B on T, C3 / C5 slices and T fp32
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_overlap.py -x -v --timeout 200 --timeout-method thread \
    > gpurun_out/overlap_tests_r5k.txt 2>&1
tail -2 gpurun_out/overlap_tests_r5k.txt
bash scripts/ab_env2.sh r5k_T 3 "--workload T" "-" "RTW_OVERLAP=2" "RTW_OVERLAP=4" "RTW_OVERLAP=8"
bash scripts/ab_env2.sh r5k_C3 2 "--workload C3 --spp 256" "-" "RTW_OVERLAP=4"
bash scripts/ab_env2.sh r5k_C5 2 "--workload C5 --spp 64" "-" "RTW_OVERLAP=4"
bash scripts/ab_env2.sh r5k_Tf 2 "--workload T --precision fp32" "-" "RTW_OVERLAP=4"
