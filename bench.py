"""bench.py — Msamples/s of the GPU render loop (the reference's "Trace" span,
RayTracingWeekend.cpp:211-250) on the north-star workload.

  python bench.py [--gpus N] [--steps K] [--warmup W]
  (N > 1: launched by torch.distributed.run, one process per GPU)

One step = one full render of the workload on every rank: rank r renders the
samples [r*spp, (r+1)*spp) of every pixel (weak scaling: the per-GPU work is
fixed as N grows), the per-pixel fp64 radiance sums are reduced to rank 0 over
RCCL, and rank 0 finalises the canvas (sum/spp, gamma 2, clamp).  Inputs (the
uploaded scene) are resident in HBM before the timed region starts.

Prints ONE JSON line on rank 0 with `roofline` (traversal kernel, algorithmic
68 B per segment over its HIP-event-timed launch durations) and `cpu_baseline`
(the reference's own code, oracle/_ref/rtw_ref, on the host cores; or the C
restatement when that binary is absent).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = json.loads((ROOT / "BASELINE.json").read_text())["metric"] if (ROOT / "BASELINE.json").exists() else \
    "Msamples/s (rays traced/s) at fixed W×H×spp×max_depth; 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
# Algorithmic bytes of the roofline kernel come from the library
# (rtw_stats.bytes_intersect = 68 B per traversal: ray 56 B in, hit 12 B out,
# SURVEY.md 8(d)).  The default kernel, k_persist, fuses traversal and
# shading and keeps the path in registers, so these bytes never actually
# reach HBM: the kernel is fp64-VALU / latency bound.


# fp64 VALU issue peak: 1024 SIMDs x 2.4 GHz / 4 cycles per wave64 instruction
VALU_PEAK_GINST = 1024 * 2.4 / 4


def workload_name(args) -> str:
    name = f"{args.scene} {args.nx}x{args.ny} {args.spp}spp/GPU max_depth {args.depth}" + (" bvh" if args.bvh else "")
    if (args.scene, args.nx, args.ny, args.spp, args.depth, args.bvh) == ("cornell_box", 800, 800, 1024, 50, False):
        name += " (north-star target T)"
    return name


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--scene", default="cornell_box")
    ap.add_argument("--nx", type=int, default=800)
    ap.add_argument("--ny", type=int, default=800)
    ap.add_argument("--spp", type=int, default=1024, help="samples per pixel per GPU")
    ap.add_argument("--depth", type=int, default=50)
    ap.add_argument("--bvh", action="store_true")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--paths", type=int, default=0, help="wavefront paths in flight (0 = library default)")
    ap.add_argument("--no-kernel-times", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-spp", type=int, default=0, help="CPU baseline sample: spp of the full image (0 = auto)")
    ap.add_argument("--ppm", default="", help="write the rank-0 canvas of the last step here")
    return ap.parse_args()


def cpu_baseline(args, threads: int):
    """Time the reference's own code (oracle/_ref/rtw_ref) -- or, when absent,
    the C restatement -- on a bounded sample of the same workload."""
    spp = args.cpu_spp or 32
    ref = ROOT / "oracle" / "_ref" / "rtw_ref"
    sample = f"{args.scene} {args.nx}x{args.ny}x{spp}spp depth {args.depth} (full image, {spp} of the workload's spp)"
    if ref.exists():
        t0 = time.perf_counter()
        r = subprocess.run([str(ref), "bench", args.scene, str(args.nx), str(args.ny), str(spp), str(args.depth),
                            str(args.seed), str(threads)], capture_output=True, text=True, timeout=600)
        wall = time.perf_counter() - t0
        if r.returncode == 0:
            info = json.loads(r.stdout.strip().splitlines()[-1])
            return {"value": round(info["msamples_per_s"], 4), "unit": "Msamples/s", "cores": threads,
                    "kind": "reference", "sample": sample, "seconds": round(info["seconds"], 3),
                    "wall_seconds": round(wall, 3),
                    "note": "reference hittable/material/pdf/camera/scene code compiled from its sources with g++ "
                            "-O2, per-path RNG injection, OpenMP over rows in place of ppl parallel_for"}
    sys.path.insert(0, str(ROOT / "tests"))
    from oracle_lib import oracle_sums
    from raytracingweekend_amd.render import SceneDesc
    sd = SceneDesc(args.scene, args.nx / args.ny, False)
    t0 = time.perf_counter()
    _, seg = oracle_sums(sd, args.nx, args.ny, spp, args.depth, args.seed, threads=threads)
    dt = time.perf_counter() - t0
    return {"value": round(args.nx * args.ny * spp / dt / 1e6, 4), "unit": "Msamples/s", "cores": threads,
            "kind": "port", "sample": sample, "seconds": round(dt, 3)}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")

    import torch
    import torch.distributed as dist
    from raytracingweekend_amd import build
    from raytracingweekend_amd.render import DeviceScene, SceneDesc, write_ppm

    if not (ROOT / "raytracingweekend_amd" / "librtw.so").exists():
        build.build_library()
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    nx, ny, spp, depth = args.nx, args.ny, args.spp, args.depth
    total_spp = spp * world
    sd = SceneDesc(args.scene, nx / ny, args.bvh)
    ds = DeviceScene(sd, local_rank)
    accum = torch.zeros(nx * ny * 3, dtype=torch.float64, device=dev)
    canvas = torch.zeros_like(accum)
    collect = not args.no_kernel_times

    def step(timed: bool):
        # one render of the workload: radiance sums on every rank, reduced to
        # rank 0, finalised to the canvas there (RayTracingWeekend.cpp:211-250);
        # the canvas stays in HBM like the inputs
        accum.zero_()
        _, st = ds.render_accumulate(nx, ny, total_spp, depth, args.seed, spp_begin=rank * spp, spp_count=spp,
                                     accum=accum, collect_kernel_times=collect and timed,
                                     wavefront_paths=args.paths)
        if world > 1:
            dist.reduce(accum, dst=0)
        if rank == 0:
            ds.finalize_device(accum, nx, ny, total_spp, canvas)
        return st, canvas

    for _ in range(args.warmup):
        step(False)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    stats = []
    canvas = None
    for _ in range(args.steps):
        st, canvas = step(True)
        stats.append(st)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    samples_per_step = nx * ny * spp * world
    seg = sum(s["segments"] for s in stats)
    ms_isect = sum(s["ms_intersect"] for s in stats)
    launches = sum(s["launches_intersect"] for s in stats)
    algo = sum(s["bytes_intersect"] for s in stats)
    mode = os.environ.get("RTW_MODE", "persistent")
    sort_env = os.environ.get("RTW_SORT", "")
    sorted_pk = sort_env == "1" or (sort_env != "0" and not args.bvh)  # the library's default (launch_pk)
    kernel = ("k_intersect" if os.environ.get("RTW_SPLIT") == "1" else "k_segment") if mode == "wavefront" \
        else ("k_persist_sort" if sorted_pk else "k_persist")
    if world > 1:
        v = torch.tensor([seg, ms_isect, launches, algo], dtype=torch.float64, device=dev)
        dist.all_reduce(v)
        seg_all, ms_all, launches_all, algo_all = float(v[0]), float(v[1]), float(v[2]), float(v[3])
    else:
        seg_all, ms_all, launches_all, algo_all = float(seg), ms_isect, float(launches), algo

    if rank == 0:
        value = samples_per_step * args.steps / elapsed / 1e6
        roofline = None
        if collect and ms_all > 0:
            achieved = algo_all / (ms_all * 1e-3) / 1e9
            traffic, valu = None, None
            pmc = ROOT / "profiles" / "pmc_intersect.json"
            workload = workload_name(args)
            if pmc.exists():
                try:
                    p = json.loads(pmc.read_text())
                except ValueError:
                    p = {}
                # PMC figures only describe the workload (and kernel) they were taken on
                if p.get("workload") == workload and p.get("kernel") == kernel:
                    # per launch, scaled from the profiled launches by traversals
                    scale = (seg_all / max(launches_all, 1)) / p["segments_per_launch"]
                    traffic = round(p["hbm_bytes_per_launch"] * scale, 1)
                    ipw = p.get("valu_insts_per_wave_segment")
                    if ipw:
                        ach = ipw * seg_all / 64 / (ms_all * 1e-3) / 1e9
                        valu = {"bound": "valu", "achieved": round(ach, 1), "peak": VALU_PEAK_GINST,
                                "unit": "G wave-instr/s", "frac": round(ach / VALU_PEAK_GINST, 4),
                                "insts_per_wave_segment": round(ipw, 1),
                                "source": "profiles/pmc_intersect.json (SQ_INSTS_VALU)"}
            roofline = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                        "kernel": kernel, "launches": int(launches_all),
                        "avg_launch_ms": round(ms_all / max(launches_all, 1), 4),
                        "algo_bytes_per_launch": round(algo_all / max(launches_all, 1), 1),
                        "bytes_per_segment": round(algo_all / max(seg_all, 1), 2)}
            if valu:
                roofline["valu"] = valu
        out = {
            "metric": METRIC, "value": round(value, 3), "unit": "Msamples/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic",
            "config": {"workload": workload_name(args),
                       "scene": args.scene, "nx": nx, "ny": ny, "spp_per_gpu": spp, "max_depth": depth,
                       "bvh": args.bvh, "parallelism": f"spp-shard x{world} + RCCL reduce"},
            "msegments_per_s": round(seg_all / args.steps / (elapsed / args.steps) / 1e6, 2) if seg_all else None,
            "segments_per_sample": round(seg_all / (samples_per_step * args.steps), 4),
            "ms_render_gpu": round(sum(s["ms_total"] for s in stats) / len(stats), 3),
            "roofline": roofline,
            "cpu_baseline": None,
        }
        if world == 1 and not args.no_cpu_baseline:
            threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
            try:
                out["cpu_baseline"] = cpu_baseline(args, threads)
            except Exception as e:  # reported, never fatal for the GPU number
                out["cpu_baseline"] = {"error": repr(e)}
        if args.ppm:
            write_ppm(args.ppm, canvas.cpu().numpy(), nx, ny)
        print(json.dumps(out), flush=True)
    ds.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
