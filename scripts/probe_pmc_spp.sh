set -e
mkdir -p gpurun_out
scripts/pmc_passes.sh T_probe --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_T_probe.log 2>&1
for s in 1024 128; do
  timeout -k 10 300 python bench.py --spp $s --steps 3 --warmup 1 --no-cpu-baseline | tail -1 | cut -c1-400 >> gpurun_out/spp_scan.txt
done
cat gpurun_out/spp_scan.txt
