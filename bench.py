"""bench.py — Msamples/s of the GPU render loop (the reference's "Trace" span,
RayTracingWeekend.cpp:211-250) on the BASELINE.json workloads.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload T|C4|C2|C3|C5|C1]
                  [--scaling strong|weak]

--gpus N > 1 runs one process per GPU: under torch.distributed.run (the
driver's launch: RANK / WORLD_SIZE / LOCAL_RANK in the environment), or, when
started directly, bench.py starts torch.distributed.run itself as a child
process (before anything touches the GPU) and exits with its status.

One step = one full render of the workload's image: rank r renders its shard
of the samples of every pixel (raytracingweekend_amd.distributed.render_step,
the same step tests/test_distributed.py runs over gloo), the per-pixel fp64
radiance sums are reduced to rank 0 over RCCL, and rank 0 finalises the canvas
on the GPU (sum/spp, gamma 2, clamp).  The scene is resident in HBM before the
timed region; the canvas stays in HBM.

Scaling: "strong" (default) keeps the workload's total samples per pixel and
splits them over the ranks -- T is 1024 spp whatever N, as the metric reads
("at fixed W x H x spp x max_depth; 1/2/4/8 GPU"); "weak" renders --spp per
GPU.  value = all samples of a step / the step's time (max over ranks).

Prints ONE JSON line on rank 0 with `rank_phases_ms` (each rank's traversal
kernel, render, RCCL reduce and finalize time per step, max / min over the
ranks and rank 0's, for diagnosing an N > 1 run), `roofline` for the traversal kernel the
library actually launched (rtw_scene_query names it): HIP-event-timed launch
durations; the VALU roofline (the binding resource) from the
PMC record of that kernel, build and workload when one is committed under
profiles/pmc/, else the §8(d) HBM figure alone; and `cpu_baseline` (the
reference's own code, oracle/_ref/rtw_ref, on the host cores; or the C
restatement when that binary is absent).
"""
from __future__ import annotations

import argparse
import datetime
import json
import os
import socket
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = json.loads((ROOT / "BASELINE.json").read_text())["metric"] if (ROOT / "BASELINE.json").exists() else \
    "Msamples/s (rays traced/s) at fixed W×H×spp×max_depth; 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
# VALU issue cycles available: 256 CUs x 4 SIMDs x 2.4 GHz
VALU_SIMD_GCYC = 1024 * 2.4
# fp64 vector peak: 1024 SIMDs x 2.4 GHz x 32 FLOP/cycle (16 fp64 FMA lanes)
FP64_PEAK_TFLOPS = 78.6
FP32_PEAK_TFLOPS = 157.3
# Issue cost of one wave64 VALU instruction per SIMD, in cycles at the nominal
# 2.4 GHz, per SQ_INSTS_VALU_* class: measured on the card with independent
# chains at 4 waves/SIMD (scripts/valu_rates.hip; profiles/r01/valu_rates.log,
# profiles/r04/valu_rates.log).  Each class takes the cheapest measured cost
# of any of its members in either log (F64: v_fma/mul/add_f64 4.59-4.81;
# TRANS_F64: v_sqrt_f64 16.35, v_rsq/rcp_f64 16.6-17.4; INT32: v_add_u32 /
# v_and_b32 / v_mov_b32 2.55-2.64, v_lshlrev / v_bfe / v_mul_lo 4.3-4.4;
# INT64: v_mad_u64_u32 5.15; CVT: v_cvt_f64_u32 5.26, v_cvt_f32_f64 5.33;
# F32: v_add_f32 2.60, v_fma_f32 2.70, packed 4.4-4.8; TRANS_F32:
# v_rcp/v_sqrt/v_exp/v_sin_f32 8.36-8.63), and instructions no class counts
# (moves, compares, selects, logic: 2.6-4.5) take the cheapest rate of all
# -- so the class-weighted cycles are a LOWER bound of the SIMDs' VALU issue
# time, and their fraction of the SIMD cycles is at most 1.
VALU_COST = {"FMA_F64": 4.59, "MUL_F64": 4.59, "ADD_F64": 4.59, "TRANS_F64": 16.35,
             "INT32": 2.55, "INT64": 5.15, "CVT": 5.26,
             "FMA_F32": 2.60, "ADD_F32": 2.60, "MUL_F32": 2.60, "TRANS_F32": 8.36}
VALU_COST_OTHER = 2.55
PMC_DIR = ROOT / "profiles" / "pmc"
# Process-group timeout: a rank stuck in a collective (or a rank that never
# joins) ends the run with a per-rank error after this many seconds instead of
# holding the driver's whole time limit.
PG_TIMEOUT_S = float(os.environ.get("RTW_BENCH_PG_TIMEOUT", "240"))

# BASELINE.json configs; spp is the image's TOTAL samples per pixel
WORKLOADS = {
    "T": dict(scene="cornell_box", nx=800, ny=800, spp=1024, depth=50, bvh=False,
              label="T: Cornell box 800x800x1024spp depth 50 (north-star target)"),
    "C4": dict(scene="cornell_box", nx=800, ny=800, spp=4096, depth=50, bvh=False,
               label="C4: Cornell box 800x800x4096spp depth 50"),
    "C2": dict(scene="random_balls", nx=1200, ny=800, spp=256, depth=50, bvh=False,
               label="C2: Book-1 random_balls 1200x800x256spp depth 50, flat list"),
    "C3": dict(scene="random_balls", nx=1200, ny=800, spp=1024, depth=50, bvh=True,
               label="C3: Book-1 random_balls + BVH 1200x800x1024spp depth 50"),
    "C5": dict(scene="book2_final", nx=1600, ny=1600, spp=4096, depth=50, bvh=True,
               label="C5: Book-2 final scene + BVH 1600x1600x4096spp depth 50"),
    "C1": dict(scene="random_balls", nx=200, ny=100, spp=16, depth=50, bvh=False,
               label="C1: Book-1 random_balls 200x100x16spp depth 50"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", default="T", choices=sorted(WORKLOADS))
    ap.add_argument("--scaling", default="strong", choices=["strong", "weak"])
    ap.add_argument("--scene", default=None, help="override the workload's scene (workload becomes custom)")
    ap.add_argument("--nx", type=int, default=None)
    ap.add_argument("--ny", type=int, default=None)
    ap.add_argument("--spp", type=int, default=None,
                    help="samples per pixel: of the whole image (strong) or per GPU (weak)")
    ap.add_argument("--depth", type=int, default=None)
    ap.add_argument("--bvh", action="store_true", default=None)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--precision", default="fp64", choices=["fp64", "fp32"],
                    help="fp64: the reference's double arithmetic (parity mode, the headline); fp32: the fast "
                         "mode, statistical parity only, reported as its own line")
    ap.add_argument("--paths", type=int, default=0, help="wavefront paths in flight (0 = library default)")
    ap.add_argument("--no-kernel-times", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-spp", type=int, default=0, help="CPU baseline sample: spp of the full image (0 = auto)")
    ap.add_argument("--ppm", default="", help="write the rank-0 canvas of the last step here")
    a = ap.parse_args()
    w = dict(WORKLOADS[a.workload])
    custom = False
    for k in ("scene", "nx", "ny", "spp", "depth", "bvh"):
        v = getattr(a, k)
        if v is not None and v != w[k]:
            w[k] = v
            custom = True
        setattr(a, k, w[k])
    a.workload_key = "custom" if custom else a.workload
    a.label = (f"custom: {a.scene} {a.nx}x{a.ny}x{a.spp}spp depth {a.depth}" + (" bvh" if a.bvh else "")) \
        if custom else w["label"]
    return a


def pmc_key(args) -> str:
    """What a PMC record must have been taken on: per-segment instruction
    counts and per-launch bytes depend on the scene, image, depth and
    precision (spp and GPU count only scale them)."""
    return (f"{args.scene} {args.nx}x{args.ny} depth {args.depth}" + (" bvh" if args.bvh else "") +
            (" fp32" if getattr(args, "precision", "fp64") == "fp32" else ""))


def find_pmc(kernel: str, build: str, key: str, pmc_dir: Path = PMC_DIR):
    """The committed PMC record for exactly this kernel, build and workload
    (profiles/pmc/*.json), or None -- a record of another build is never used."""
    if not pmc_dir.is_dir():
        return None, "no profiles/pmc directory"
    seen = []
    for f in sorted(pmc_dir.glob("*.json")):
        try:
            p = json.loads(f.read_text())
        except ValueError:
            continue
        if p.get("kernel") == kernel and p.get("build_id") == build and p.get("workload") == key:
            return p, f.name
        seen.append(f"{f.name}: {p.get('kernel')} / {p.get('build_id')} / {p.get('workload')}")
    return None, "no PMC record for this kernel / build / workload (" + "; ".join(seen) + ")"


# Bounded CPU sample per scene, (spp, row stride): about 10-20 s of the
# reference's code on the GPU box's 16 host threads (Cornell ~1.4, random_balls
# ~0.15, Book-2 final ~0.015 Msamples/s there).
CPU_SAMPLE = {"cornell_box": (32, 1), "random_balls": (16, 8), "book2_final": (4, 16)}


def cpu_baseline(args, threads: int, use_reference: bool = True):
    """Time the reference's own code (oracle/_ref/rtw_ref) -- or, when absent,
    the C restatement -- on a bounded sample of the same workload: every
    `stride`-th row of the image at `spp` samples per pixel."""
    spp, stride = CPU_SAMPLE.get(args.scene, (8, 1))
    spp = args.cpu_spp or spp
    rows = list(range(0, args.ny, stride))
    ref = ROOT / "oracle" / "_ref" / "rtw_ref"
    sample = (f"{args.scene} {args.nx}x{args.ny} depth {args.depth}: {spp} spp of "
              + ("every row" if stride == 1 else f"every {stride}th row ({len(rows)} of {args.ny})"))
    if use_reference and ref.exists():
        t0 = time.perf_counter()
        r = subprocess.run([str(ref), "bench", args.scene, str(args.nx), str(args.ny), str(spp), str(args.depth),
                            str(args.seed), str(threads), str(stride)], capture_output=True, text=True, timeout=600)
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
    # one call over the strided rows: OpenMP spreads them over `threads`
    oracle_sums(sd, args.nx, args.ny, spp, args.depth, args.seed, threads=threads, rows=(0, len(rows), stride))
    dt = time.perf_counter() - t0
    return {"value": round(args.nx * len(rows) * spp / dt / 1e6, 4), "unit": "Msamples/s", "cores": threads,
            "kind": "port", "sample": sample, "seconds": round(dt, 3)}


def spawn(args) -> int:
    """Start torch.distributed.run with one rank per GPU (child process; this
    process never touches the GPU) and return its exit status."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", str(Path(__file__).resolve()), *sys.argv[1:]]
    return subprocess.call(cmd, env={**os.environ, "HSA_ENABLE_IPC_MODE_LEGACY": "0"})


def roofline(args, kernel, build, seg, ms, launches, algo, check=True):
    """Roofline object of the traversal kernel (per launch averages).

    The headline (bound / achieved / peak / frac) is SURVEY.md 8(d)'s HBM
    figure: 68 algorithmic bytes per traversal (36 in fp32) x device-counted
    traversals / HIP-event launch time, against 8 TB/s; `traffic` = the HBM
    bytes the PMC record of this kernel, build and workload measured.  Beside
    it, `valu` (from the same record): (i) class-weighted VALU issue cycles
    over the SIMDs' cycles, (ii) the fp64 FLOP rate against the vector peak,
    and the lane utilisation.  Every fraction is bounded by 1 (checked)."""
    avg_ms = ms / max(launches, 1)
    seg_launch = seg / max(launches, 1)
    hbm_ach = algo / (ms * 1e-3) / 1e9
    out = {"kernel": kernel, "build_id": build, "launches": int(launches), "avg_launch_ms": round(avg_ms, 4),
           "segments_per_launch": round(seg_launch, 1),
           "bound": "hbm", "achieved": round(hbm_ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(hbm_ach / HBM_PEAK_GBS, 4), "traffic": None,
           "bytes_per_segment": round(algo / max(seg, 1), 2),
           "algo_bytes_per_launch": round(algo / max(launches, 1), 1),
           "definition": "SURVEY.md 8(d): 68 algorithmic bytes per traversal in fp64 (ray 56 B in, hit 12 B out; "
                         "36 B in the fp32 fast mode) x device-counted traversals / HIP-event launch time, against "
                         "8 TB/s; traffic = PMC FETCH_SIZE + WRITE_SIZE bytes per launch of the same kernel and build"}
    rec, src = find_pmc(kernel, build, pmc_key(args))
    out["pmc"] = src
    if rec is None:
        return out
    scale = seg_launch / rec["segments_per_launch"]  # PMC bytes per launch, scaled by traversals
    out["traffic"] = round(rec["hbm_bytes_per_launch"] * scale, 1)
    if rec.get("write_bytes_per_launch") is not None:
        out["write_bytes"] = round(rec["write_bytes_per_launch"] * scale, 1)
    secs = avg_ms * 1e-3
    if rec.get("clock_ghz_x_ms") and rec.get("avg_launch_ms"):
        # the clock the record's launches ran at (GRBM busy cycles / launch time): the peaks
        # below assume 2.4 GHz; a power-limited box runs some workloads slower
        out["pmc_clock_ghz"] = round(rec["clock_ghz_x_ms"] / rec["avg_launch_ms"], 3)
    v = {"valu_insts_per_wave_segment": round(rec["valu_insts_per_wave_segment"], 1),
         "lane_util": round(rec["valu_lane_util"], 4) if rec.get("valu_lane_util") else None}
    cyc = rec.get("valu_class_cycles_per_segment")
    if cyc:
        ach = cyc * seg_launch / secs / 1e9
        v["class_weighted"] = {
            "achieved": round(ach, 1), "peak": VALU_SIMD_GCYC, "unit": "G SIMD-cycles/s",
            "frac": round(ach / VALU_SIMD_GCYC, 4), "cycles_per_segment": round(cyc, 2),
            "definition": "SQ_INSTS_VALU_{FMA,MUL,ADD,TRANS}_F64, _INT32, _INT64, _CVT, _{FMA,ADD,MUL,TRANS}_F32 "
                          "x their measured issue cycles (VALU_COST), unclassified VALU at the cheapest rate, per "
                          "traversal of the PMC record x this run's traversals / launch time, against 1024 SIMDs "
                          "x 2.4 GHz (a lower bound of VALU issue time)"}
        if v["lane_util"]:
            v["useful_frac"] = round(ach / VALU_SIMD_GCYC * v["lane_util"], 4)
    lane = v["lane_util"] or 1.0
    fl = rec.get("fp64_flops_per_segment")
    if fl is not None:
        issued = fl * seg_launch / secs / 1e12
        v["fp64_flops"] = {"achieved": round(issued * lane, 3), "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                           "frac": round(issued * lane / FP64_PEAK_TFLOPS, 4), "issued": round(issued, 3),
                           "issued_frac": round(issued / FP64_PEAK_TFLOPS, 4),
                           "definition": "SQ_INSTS_VALU_FLOPS_FP64 (per wave instruction: FMA 2, MUL / ADD / TRANS "
                                         "1) x 64 lanes per traversal x traversals / launch time = issued; x the lane "
                                         "utilisation = achieved; against the 78.6 TF fp64 vector peak"}
    fl32 = rec.get("fp32_flops_per_segment")
    if fl32:
        issued = fl32 * seg_launch / secs / 1e12
        v["fp32_flops"] = {"achieved": round(issued * lane, 3), "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                           "frac": round(issued * lane / FP32_PEAK_TFLOPS, 4), "issued": round(issued, 3)}
    out["valu"] = v
    if check:
        check_fracs(out)
    return out


def check_fracs(obj, path="roofline"):
    """Every `frac` of a roofline object is a fraction of a peak: in [0, 1]."""
    if isinstance(obj, dict):
        for k, val in obj.items():
            if k == "frac" and not (0.0 <= val <= 1.0):
                raise ValueError(f"{path}.frac = {val} is not a roofline fraction")
            check_fracs(val, f"{path}.{k}")


def bounded_valu(out):
    """check_fracs for the bench line: a VALU fraction above 1 (e.g. a PMC
    record slightly stale against this run's launch time) drops the `valu`
    sub-object and leaves a warning in the line instead of aborting before
    the result is printed (tests/test_bench.py keeps the hard check)."""
    try:
        check_fracs(out)
    except ValueError as e:
        out.pop("valu", None)
        out["warning"] = f"valu figures dropped: {e}"
    return out


# Per-rank phase times of the timed steps (ms per step): the traversal
# kernel's HIP-event time, and render_step's wall phases (render = zero +
# render call incl. k_reduce / k_emit, reduce = the RCCL collective,
# finalize = rank 0's device finalize).
RANK_PHASES = ("kernel", "render", "reduce", "finalize")


def rank_phases(local: dict, world: int, device=None) -> dict:
    """{phase: {"max", "min", "rank0"}} over the ranks, reduced with
    all_reduce MAX / MIN as the step time is (the rank-0 value broadcast from
    rank 0).  world == 1: all three are this rank's value."""
    vals = [float(local.get(k, 0.0)) for k in RANK_PHASES]
    if world > 1:
        import torch
        import torch.distributed as dist
        hi = torch.tensor(vals, dtype=torch.float64, device=device)
        lo = hi.clone()
        r0 = hi.clone()
        dist.all_reduce(hi, op=dist.ReduceOp.MAX)
        dist.all_reduce(lo, op=dist.ReduceOp.MIN)
        dist.broadcast(r0, src=0)
        mx, mn, z = hi.tolist(), lo.tolist(), r0.tolist()
    else:
        mx = mn = z = vals
    return {k: {"max": round(mx[i], 3), "min": round(mn[i], 3), "rank0": round(z[i], 3)}
            for i, k in enumerate(RANK_PHASES)}


def device_record(gpu: int) -> dict:
    """What this rank runs on: the HIP device index and the card's PCI
    address (domain:bus:device, as rocm-smi prints it) and name."""
    import torch
    p = torch.cuda.get_device_properties(gpu)
    return {"device": gpu, "pci_bus_id": f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}",
            "name": p.name, "arch": getattr(p, "gcnArchName", "")}


def rank_devices(world: int, rank: int, local_rank: int, dev_rec: dict) -> dict:
    """The line's record of who ran where: every rank's {rank, local_rank,
    device, pci_bus_id, ...} gathered over the process group
    (all_gather_object), the group's backend and world size, and how many
    distinct cards the ranks used -- so an N > 1 line shows by itself whether
    RCCL saw N ranks on N distinct devices."""
    me = {"rank": rank, "local_rank": local_rank, **dev_rec}
    if world > 1:
        import torch.distributed as dist
        ranks = [None] * world
        dist.all_gather_object(ranks, me)
        backend = dist.get_backend()
        size = dist.get_world_size()
    else:
        ranks, backend, size = [me], None, 1
    ranks = sorted(ranks, key=lambda r: r["rank"])
    return {"process_group": {"backend": backend, "world_size": size, "timeout_s": PG_TIMEOUT_S if world > 1 else None},
            "ranks": ranks, "distinct_devices": len({r.get("pci_bus_id") for r in ranks})}


def result_line(args, world, spp_total, elapsed, samples, seg, ms_gpu, roof, phases, placement=None) -> dict:
    """The rank-0 JSON line (the driver's contract): value = all samples of
    the timed steps / the step time (max over ranks)."""
    samples_per_step = args.nx * args.ny * spp_total
    assert int(samples) == samples_per_step * args.steps, "ranks rendered a different number of samples"
    value = samples_per_step * args.steps / elapsed / 1e6
    return {
        "metric": METRIC, "value": round(value, 3), "unit": "Msamples/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": args.scaling, "vs_baseline": None,
        "dtype": "f32" if args.precision == "fp32" else "f64",
        "data": "synthetic (the reference's own scene definitions, seeded RNG)",
        "config": {"workload": args.label, "workload_id": args.workload_key, "scene": args.scene, "nx": args.nx,
                   "ny": args.ny, "spp_total": spp_total, "spp_per_gpu": spp_total / world,
                   "max_depth": args.depth, "bvh": args.bvh, "precision": args.precision,
                   "global_batch": samples_per_step,
                   "parallelism": f"spp-shard x{world}" + (
                       (" + gloo reduce (rehearsal: every rank on cuda:0)" if getattr(args, "shared_gpu", False)
                        else " + RCCL reduce") if world > 1 else "")},
        "msegments_per_s": round(seg / elapsed / 1e6, 2) if seg else None,
        "segments_per_sample": round(seg / max(samples, 1), 4),
        "ms_render_gpu": round(ms_gpu, 3),
        "roofline": roof,
        # per-rank ms per step, max / min over the ranks and rank 0's own
        # (a slow rank, the RCCL reduce and the finalize in an N > 1 run)
        "rank_phases_ms": phases,
        # every rank's device and the process group (rank_devices)
        **(placement or {}),
        "cpu_baseline": None,
    }


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn(args))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    import torch.distributed as dist
    from raytracingweekend_amd import build
    from raytracingweekend_amd.distributed import gpu_finalize_fn, gpu_render_fn, render_step
    from raytracingweekend_amd.render import DeviceScene, SceneDesc, write_ppm

    if not (ROOT / "raytracingweekend_amd" / "librtw.so").exists():
        build.build_library()
    # RTW_BENCH_SHARED_GPU=1: a rehearsal of the N > 1 path on a one-GPU box --
    # every rank renders on cuda:0 and the collectives run over gloo (RCCL
    # refuses two ranks on one device).  Its line says so in config.parallelism.
    args.shared_gpu = world > 1 and os.environ.get("RTW_BENCH_SHARED_GPU", "") == "1"
    gpu = 0 if args.shared_gpu else local_rank
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    if world > 1:
        timeout = datetime.timedelta(seconds=PG_TIMEOUT_S)
        if args.shared_gpu:
            dist.init_process_group("gloo", timeout=timeout)
        else:
            dist.init_process_group("nccl", device_id=dev, timeout=timeout)
    placement = rank_devices(world, rank, local_rank, device_record(gpu))

    nx, ny, depth = args.nx, args.ny, args.depth
    spp_total = args.spp if args.scaling == "strong" else args.spp * world
    sd = SceneDesc(args.scene, nx / ny, args.bvh)
    ds = DeviceScene(sd, gpu)
    info = ds.query()
    accum = torch.zeros(nx * ny * 3, dtype=torch.float64, device=dev)
    canvas = torch.zeros_like(accum)
    collect = not args.no_kernel_times

    phase_ms = {}  # this rank's render / reduce / finalize wall ms over the timed steps

    def step(timed: bool):
        fn = gpu_render_fn(ds, nx, ny, spp_total, depth, args.seed, collect_kernel_times=collect and timed,
                           wavefront_paths=args.paths, precision=args.precision)
        return render_step(fn, gpu_finalize_fn(ds, nx, ny, spp_total), accum, canvas, nx, ny, spp_total,
                           timings=phase_ms if timed else None, sync=torch.cuda.synchronize)

    for _ in range(args.warmup):
        step(False)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    stats = []
    for _ in range(args.steps):
        st = step(True)
        if st:
            stats.append(st)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    seg = sum(s["segments"] for s in stats)
    ms_isect = sum(s["ms_intersect"] for s in stats)
    launches = sum(s["launches_intersect"] for s in stats)
    algo = sum(s["bytes_intersect"] for s in stats)
    samples = sum(s["samples"] for s in stats)
    local = {k: v / max(args.steps, 1) for k, v in phase_ms.items()}
    local["kernel"] = ms_isect / max(args.steps, 1)
    phases = rank_phases(local, world, dev)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        v = torch.tensor([seg, ms_isect, launches, algo, samples], dtype=torch.float64, device=dev)
        dist.all_reduce(v)
        seg, ms_isect, launches, algo, samples = (float(x) for x in v.tolist())

    if rank == 0:
        kernel = info["kernel_fast"] if args.precision == "fp32" else info["kernel"]
        roof = bounded_valu(roofline(args, kernel, info["build_id"], seg, ms_isect, launches, algo, check=False)) \
            if collect and ms_isect > 0 else None
        if roof:
            roof["bvh_lds_nodes"] = info["bvh_lds_nodes"]  # BVH node packet staged in LDS per workgroup
        ms_gpu = sum(s["ms_total"] for s in stats) / max(len(stats), 1)
        out = result_line(args, world, spp_total, elapsed, samples, seg, ms_gpu, roof, phases, placement)
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
