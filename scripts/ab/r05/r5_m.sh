#!/bin/bash
# round 5, call m: magic-number sample decomposition + device reciprocals of
# nx, ny in camera_sample (in-tree build, with the DPP prefix) -- GPU suite,
# bit-identity against librtw_dpp (the DPP prefix alone), then A/B
set -e
B=raytracingweekend_amd/_build
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/gpu_tests_r5m.txt 2>&1 || { tail -30 gpurun_out/gpu_tests_r5m.txt; exit 1; }
tail -1 gpurun_out/gpu_tests_r5m.txt
timeout -k 10 300 python scripts/lib_parity.py $B/librtw_dpp.so | tee gpurun_out/parity_r5m.log
timeout -k 10 300 python scripts/lib_parity.py --fp32 $B/librtw_dpp.so cornell_box book2_final | tee -a gpurun_out/parity_r5m.log
bash scripts/ab_libs.sh r5m_T 3 "--workload T" default $B/librtw_dpp.so
bash scripts/ab_libs.sh r5m_C3 2 "--workload C3 --spp 256" default $B/librtw_dpp.so
bash scripts/ab_libs.sh r5m_C5 2 "--workload C5 --spp 64" default $B/librtw_dpp.so
bash scripts/ab_libs.sh r5m_Tf 2 "--workload T --precision fp32" default $B/librtw_dpp.so
