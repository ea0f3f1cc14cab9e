#!/bin/bash
# round 5, call f: BVH leaf sizes (runtime, RTW_BVH_LEAF_MAX for group BVHs,
# RTW_BVH_WORLD_LEAF_MAX for the world BVH) on C5 / C3 slices
set -e
bash scripts/ab_env2.sh r5f_leaf 2 "--workload C5 --spp 64" - "RTW_BVH_LEAF_MAX=1" "RTW_BVH_LEAF_MAX=3"
bash scripts/ab_env2.sh r5f_leaf 2 "--workload C3 --spp 256" - "RTW_BVH_WORLD_LEAF_MAX=2"
