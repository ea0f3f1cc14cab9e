#!/bin/bash
# PMC counters of a short bench run (kernel-trace only; no sys/runtime trace).
# Usage: scripts/prof_pmc.sh <tag> "<counters>" [bench args...]
set -e
tag=$1; shift
counters=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 rocprofv3 --kernel-trace --pmc $counters -d "gpurun_out/pmc_$tag" -o run --output-format csv -- \
    python3 bench.py "$@" > "gpurun_out/pmc_$tag.log" 2>&1
