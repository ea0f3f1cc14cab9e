#!/bin/bash
# round 5 evidence, part 2 (tag $1): PMC records of the fp32 workloads, then
# (records in profiles/pmc/ first, so the lines carry them) the default T
# line with its CPU baseline, the config lines, the fp32 lines and the
# full-size C4 / C5 lines
set -e
tag=$1
mkdir -p gpurun_out profiles/pmc
for w in "Tfp32_$tag" "C2fp32_$tag --workload C2" "C3fp32_$tag --workload C3" "C5fp32_$tag --workload C5 --spp 64"; do
    set -- $w
    t=$1; shift
    scripts/pmc_passes.sh $t "$@" --precision fp32 --steps 2 --warmup 1 --no-cpu-baseline
    echo "pmc $t done"
done
cp gpurun_out/pmc/*_$tag.json profiles/pmc/
timeout -k 10 300 python bench.py > gpurun_out/bench_T_$tag.txt 2>&1
tail -n 1 gpurun_out/bench_T_$tag.txt | cut -c1-300
bash scripts/bench_configs.sh $tag > /dev/null
bash scripts/bench_fp32.sh $tag > /dev/null
bash scripts/full_configs.sh $tag > /dev/null
