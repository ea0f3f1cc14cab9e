#!/bin/bash
# PMC records (profiles/pmc/ keyed by kernel, build and workload) for the
# single-GPU workloads: T, C2, C3 and a C5 slice (64 of its 4096 spp: per-segment
# counts do not depend on spp), and the fp32 fast mode's T, C2, C3 and C5.
# Usage: scripts/pmc_workloads.sh <round-tag>
set -e
r=$1
scripts/pmc_passes.sh T_$r --steps 2 --warmup 1 --no-cpu-baseline
scripts/pmc_passes.sh C2_$r --workload C2 --steps 2 --warmup 1 --no-cpu-baseline
scripts/pmc_passes.sh C3_$r --workload C3 --steps 2 --warmup 1 --no-cpu-baseline
scripts/pmc_passes.sh C5_$r --workload C5 --spp 64 --steps 2 --warmup 1 --no-cpu-baseline
scripts/pmc_passes.sh Tfp32_$r --precision fp32 --steps 2 --warmup 1 --no-cpu-baseline
scripts/pmc_passes.sh C2fp32_$r --workload C2 --precision fp32 --steps 2 --warmup 1 --no-cpu-baseline
scripts/pmc_passes.sh C3fp32_$r --workload C3 --precision fp32 --steps 2 --warmup 1 --no-cpu-baseline
scripts/pmc_passes.sh C5fp32_$r --workload C5 --spp 64 --precision fp32 --steps 2 --warmup 1 --no-cpu-baseline
