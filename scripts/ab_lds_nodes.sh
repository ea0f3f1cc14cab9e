#!/bin/bash
# A/B of the BVH node packet in LDS (RTW_LDS_NODES=0 turns it off) on the BVH
# workloads C3 and a C5 slice, interleaved rounds, into gpurun_out/ab_nodes_<tag>.log.
# Usage: scripts/ab_lds_nodes.sh <tag> [rounds]
set -e
tag=$1; rounds=${2:-3}
out=gpurun_out/ab_nodes_$tag.log
mkdir -p gpurun_out; : > $out
for r in $(seq 1 "$rounds"); do
    for w in "--workload C3" "--workload C5 --spp 64"; do
        for n in default 0; do
            if [ $n = default ]; then unset RTW_LDS_NODES; else export RTW_LDS_NODES=$n; fi
            line=$(timeout -k 10 300 python bench.py $w --steps 2 --warmup 1 --no-cpu-baseline | tail -1)
            python3 -c "import json,sys; d=json.loads(sys.argv[1]); r=d['roofline']; print('round $r', d['config']['workload_id'], 'nodes', r['bvh_lds_nodes'], d['value'])" "$line" | tee -a $out
        done
    done
done
unset RTW_LDS_NODES
