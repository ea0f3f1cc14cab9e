#!/bin/bash
# A/B of box items in group BVHs (RTW_BVH_BOX_ITEMS, flattener) on a C5
# slice, interleaved rounds -> gpurun_out/ab_box_<tag>.log
# Usage: scripts/ab_box.sh <tag> <rounds>
tag=$1; rounds=$2
mkdir -p gpurun_out
for r in $(seq 1 "$rounds"); do
    for s in 1 0; do
        v=$(RTW_BVH_BOX_ITEMS=$s timeout -k 10 300 python bench.py --workload C5 --spp 64 --steps 2 --warmup 1 \
            --no-cpu-baseline | grep -o '"value": [0-9.]*')
        echo "round $r | C5 slice | RTW_BVH_BOX_ITEMS=$s | $v" | tee -a gpurun_out/ab_box_$tag.log
    done
done
