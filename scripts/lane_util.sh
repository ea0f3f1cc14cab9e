#!/bin/bash
# Lane utilisation and VALU-busy counters (the P6 group of pmc_passes.sh)
# alone, for T, C2, C3 and a C5 slice: gpurun_out/pmc_lane_<tag>_<W>/ + .log
# Usage: scripts/lane_util.sh <tag>
set -e
tag=$1
P6="SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_CVT GRBM_GUI_ACTIVE"
scripts/prof_pmc.sh "lane_${tag}_T" "$P6" --steps 1 --warmup 1 --no-cpu-baseline
scripts/prof_pmc.sh "lane_${tag}_C2" "$P6" --workload C2 --steps 1 --warmup 1 --no-cpu-baseline
scripts/prof_pmc.sh "lane_${tag}_C3" "$P6" --workload C3 --steps 1 --warmup 1 --no-cpu-baseline
scripts/prof_pmc.sh "lane_${tag}_C5" "$P6" --workload C5 --spp 64 --steps 1 --warmup 1 --no-cpu-baseline
