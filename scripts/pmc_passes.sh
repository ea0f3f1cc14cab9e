#!/bin/bash
# Instruction-mix / stall / HBM-byte counters of a short bench run, one
# rocprofv3 --pmc pass per counter group (kernel-trace only), folded into
# profiles/pmc/<tag>.json (scripts/pmc_to_json.py: kernel, build and workload
# taken from the measured bench lines).
# Usage: scripts/pmc_passes.sh <tag> [bench args...]
set -e
tag=$1; shift
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH"
P2="SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_WAVE_CYCLES"
P3="SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS"
P4="FETCH_SIZE GRBM_GUI_ACTIVE"
P5="WRITE_SIZE GRBM_COUNT"
# lane utilisation (VALUUtilization = THREAD_CYCLES_VALU / (64 ACTIVE_INST_VALU))
# and the fp32 / conversion classes of the instruction mix
P6="SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_CVT GRBM_GUI_ACTIVE"
# FLOP counts (lane-weighted) for the fp64 / fp32 FLOP rate against the vector peaks
P7="SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP64_TRANS SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FLOPS_FP32_TRANS SQ_INSTS_VALU_IOPS GRBM_GUI_ACTIVE"
i=1
dirs=()
for grp in "$P1" "$P2" "$P3" "$P4" "$P5" "$P6" "$P7"; do
    scripts/prof_pmc.sh "${tag}_$i" "$grp" "$@"
    dirs+=("gpurun_out/pmc_${tag}_$i")
    i=$((i+1))
done
python3 scripts/pmc_to_json.py "gpurun_out/pmc/${tag}.json" "${dirs[@]}"
