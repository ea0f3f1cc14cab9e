#!/bin/bash
# why are 16-B nodes slower: issue rate of v_fma_mix_f32 / v_cvt_f32_f16, and the variant with converted bounds
set -e
mkdir -p gpurun_out
timeout -k 10 60 scripts/bin/valu_rates > gpurun_out/valu_rates_r4f.log 2>&1
tail -3 gpurun_out/valu_rates_r4f.log
B=raytracingweekend_amd/_build
bash scripts/ab_libs.sh r4f 2 "--workload C3" default $B/librtw_node16.so $B/librtw_node16cvt.so
bash scripts/ab_libs.sh r4f 2 "--workload C5 --spp 64" default $B/librtw_node16.so $B/librtw_node16cvt.so
