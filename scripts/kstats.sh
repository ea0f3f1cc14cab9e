#!/bin/bash
# rocprofv3 kernel-trace stats of one short bench run per library:
# gpurun_out/kstats_<tag>_<i>/ (+ .log)
# Usage: scripts/kstats.sh <tag> "<bench args>" lib1 lib2 ...   ("default" = in-tree librtw.so)
set -e
tag=$1; args=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
i=0
for lib in "$@"; do
    if [ "$lib" = default ]; then unset RTW_LIBRARY; else export RTW_LIBRARY=$lib; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "gpurun_out/kstats_${tag}_$i" -o run --output-format csv -- \
        python3 bench.py $args --steps 1 --warmup 1 --no-cpu-baseline > "gpurun_out/kstats_${tag}_$i.log" 2>&1
    echo "== $lib"; grep -h -E "k_persist|k_reduce|k_fast" gpurun_out/kstats_${tag}_$i/run_kernel_stats.csv | cut -d, -f1-6
    i=$((i+1))
done
