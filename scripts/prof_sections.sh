set -e
mkdir -p gpurun_out
export RTW_LIBRARY=raytracingweekend_amd/_build/librtw_prof.so
timeout -k 10 200 python bench.py --spp 128 --steps 1 --warmup 0 --no-cpu-baseline --no-kernel-times > gpurun_out/prof_T.txt 2>&1
timeout -k 10 200 python bench.py --workload C3 --spp 128 --steps 1 --warmup 0 --no-cpu-baseline --no-kernel-times > gpurun_out/prof_C3.txt 2>&1
grep "rtw prof" gpurun_out/prof_T.txt gpurun_out/prof_C3.txt
