#!/bin/bash
# scripts/round_evidence.sh in three GPU calls (each under gpurun's 20-minute
# limit); outputs under gpurun_out/, copied into profiles/<round>/ and
# profiles/pmc/ afterwards.
#   scripts/evidence_parts.sh <tag> fp64    GPU suite, rocprof of the default bench command,
#                                           PMC records T, C2, C3, C5 (64-spp slice)
#   scripts/evidence_parts.sh <tag> fp32    PMC records of the fp32 fast mode's T, C2, C3, C5
#   scripts/evidence_parts.sh <tag> lines   the default bench line (T, with the CPU baseline),
#                                           the config lines, the fp32 lines and the full-size
#                                           C4 / C5 lines -- run with the PMC records of this
#                                           build already in profiles/pmc/, so every line's
#                                           roofline carries them
set -e
tag=$1
part=$2
export TMPDIR=/tmp
mkdir -p gpurun_out
case "$part" in
fp64)
    timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
        > gpurun_out/gpu_tests_$tag.txt 2>&1
    tail -1 gpurun_out/gpu_tests_$tag.txt
    scripts/prof_kernels.sh T_$tag --steps 3 --warmup 1 --no-cpu-baseline
    scripts/pmc_passes.sh T_$tag --steps 2 --warmup 1 --no-cpu-baseline
    scripts/pmc_passes.sh C2_$tag --workload C2 --steps 2 --warmup 1 --no-cpu-baseline
    scripts/pmc_passes.sh C3_$tag --workload C3 --steps 2 --warmup 1 --no-cpu-baseline
    scripts/pmc_passes.sh C5_$tag --workload C5 --spp 64 --steps 2 --warmup 1 --no-cpu-baseline
    ;;
fp32)
    scripts/pmc_passes.sh Tfp32_$tag --precision fp32 --steps 2 --warmup 1 --no-cpu-baseline
    scripts/pmc_passes.sh C2fp32_$tag --workload C2 --precision fp32 --steps 2 --warmup 1 --no-cpu-baseline
    scripts/pmc_passes.sh C3fp32_$tag --workload C3 --precision fp32 --steps 2 --warmup 1 --no-cpu-baseline
    scripts/pmc_passes.sh C5fp32_$tag --workload C5 --spp 64 --precision fp32 --steps 2 --warmup 1 \
        --no-cpu-baseline
    ;;
lines)
    timeout -k 10 300 python bench.py > gpurun_out/bench_T_$tag.txt 2>&1
    tail -1 gpurun_out/bench_T_$tag.txt | cut -c1-200
    bash scripts/bench_configs.sh $tag > /dev/null
    bash scripts/bench_fp32.sh $tag > /dev/null
    bash scripts/full_configs.sh $tag > /dev/null
    ;;
*)
    echo "unknown part $part" >&2
    exit 2
    ;;
esac
