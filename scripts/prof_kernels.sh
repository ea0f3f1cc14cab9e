#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run.  Usage: scripts/prof_kernels.sh <tag> [bench args...]
set -e
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "gpurun_out/prof_$tag" -o run --output-format csv -- \
    python3 bench.py "$@" > "gpurun_out/prof_$tag.log" 2>&1
