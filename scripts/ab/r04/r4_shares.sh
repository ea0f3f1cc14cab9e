#!/bin/bash
# The per-GPU shares of the driver's strong-scaling run, on one GPU: T (1024 / 512 / 256 / 128 spp)
# and C5 (4096 / 2048 / 1024 / 512 spp) -- what each rank renders at N = 1, 2, 4, 8
set -e
mkdir -p gpurun_out
out=gpurun_out/shares_r4q.log; : > $out
for spp in 1024 512 256 128; do
  timeout -k 10 300 python bench.py --workload T --spp $spp --steps 3 --warmup 1 --no-cpu-baseline --no-kernel-times | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('T spp', $spp, d['value'], 'ms/step', d['ms_per_step'])" | tee -a $out
done
for spp in 4096 2048 1024 512; do
  timeout -k 10 300 python bench.py --workload C5 --spp $spp --steps 1 --warmup 1 --no-cpu-baseline --no-kernel-times | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C5 spp', $spp, d['value'], 'ms/step', d['ms_per_step'])" | tee -a $out
done
