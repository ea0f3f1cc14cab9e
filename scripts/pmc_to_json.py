"""Fold the rocprofv3 --pmc passes of scripts/pmc_passes.sh into one PMC
record of the traversal kernel, keyed the way bench.py looks it up
(profiles/pmc/*.json: kernel, build_id, workload).

The kernel, its build id, the workload key and the traversals per launch come
from the bench line each pass printed (its `roofline` object), so a record
can only describe the library that was measured.

HBM bytes per launch follow MI355X_MICROARCH.md (HBM / rocprofv3): FETCH_SIZE
and WRITE_SIZE are KiB from the L2's fabric request counters, FETCH_SIZE
counted at half the bytes of wide streaming reads (x2 here), each from its own
pass.  SQ cycle counters are in units of 4 cycles.

The derived figures (`derive`) are bounded:
  * valu_class_cycles_per_segment: SIMD issue cycles of the measured
    instruction mix -- each SQ_INSTS_VALU_* class times its measured cost per
    wave64 instruction (bench.VALU_COST, profiles/r01/valu_rates.log,
    profiles/r04/valu_rates.log), the instructions no class counts (moves,
    compares, selects, logic) at the cheapest measured rate -- per traversal;
    bench.py divides by the launch time x 1024 SIMDs x clock;
  * fp64_flops_per_segment: SQ_INSTS_VALU_FLOPS_FP64 x 64 lanes per
    traversal (the counter counts per wave instruction), against the 78.6 TF
    fp64 vector peak in bench.py, issued and lane-weighted;
  * valu_lane_util: SQ_THREAD_CYCLES_VALU / (64 SQ_ACTIVE_INST_VALU).
SQ_ACTIVE_INST_VALU sums the cycles of every co-resident wave, so its ratio
to the SIMD cycles is kept only as a diagnostic (valu_active_wave_sum); it can
pass 1 and is not a roofline fraction.

Usage: python scripts/pmc_to_json.py <out.json> <pass-dir> [<pass-dir> ...]
       (each pass dir = gpurun_out/pmc_<tag>_<i>, with pmc_<tag>_<i>.log beside it)
       python scripts/pmc_to_json.py --refresh <record.json> ...
       (re-derive committed records from their raw_per_launch counters)
"""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from bench import VALU_COST, VALU_COST_OTHER, pmc_key  # noqa: E402


def bench_line(log: Path) -> dict:
    for line in reversed(log.read_text().splitlines()):
        if line.startswith("{"):
            return json.loads(line)
    raise SystemExit(f"{log}: no bench line")


def derive(per: dict, seg_per_launch: float) -> dict:
    """Every figure of a record that follows from its per-launch counters."""
    wave_segments = seg_per_launch / 64 if seg_per_launch else 0
    ws = (lambda v: v / wave_segments) if wave_segments else (lambda v: None)
    fetch = per.get("FETCH_SIZE", 0.0) * 1024 * 2
    write = per.get("WRITE_SIZE", 0.0) * 1024
    valu = per.get("SQ_INSTS_VALU", 0.0)
    classes = {k: per[f"SQ_INSTS_VALU_{k}"] for k in VALU_COST if f"SQ_INSTS_VALU_{k}" in per}
    other = max(0.0, valu - sum(classes.values()))
    # the record must hold every class (pmc_passes.sh P2 + P6 + P7); a record
    # that misses one would price its instructions at the cheapest rate
    complete = valu > 0 and all(f"SQ_INSTS_VALU_{k}" in per for k in VALU_COST)
    cycles = sum(VALU_COST[k] * v for k, v in classes.items()) + VALU_COST_OTHER * other
    # SQ_INSTS_VALU_FLOPS_FP64 counts per WAVE instruction (FMA 2, MUL / ADD /
    # TRANS 1; _TRANS is a subset): measured, it equals 2 FMA_F64 + MUL_F64 +
    # ADD_F64 + TRANS_F64 (profiles/pmc/T_r4a.json).  x 64 lanes = the FLOPs
    # the issued instructions could do with every lane on (an upper bound);
    # bench.py weights it by the lane utilisation for the useful rate.
    flops64 = per.get("SQ_INSTS_VALU_FLOPS_FP64")
    flops64 = flops64 * 64 if flops64 is not None else None
    flops32 = per.get("SQ_INSTS_VALU_FLOPS_FP32")
    flops32 = flops32 * 64 if flops32 is not None else None
    gui = per.get("GRBM_GUI_ACTIVE")
    act = per.get("SQ_ACTIVE_INST_VALU")
    cyc = per.get("SQ_WAVE_CYCLES", 0) or 1
    return {
        "hbm_bytes_per_launch": fetch + write,
        "fetch_bytes_per_launch": fetch,
        "write_bytes_per_launch": write,
        "valu_insts_per_wave_segment": ws(valu),
        "salu_insts_per_wave_segment": ws(per.get("SQ_INSTS_SALU", 0)),
        "f64_insts_per_wave_segment": {k: ws(per.get(f"SQ_INSTS_VALU_{k}", 0))
                                       for k in ("FMA_F64", "MUL_F64", "ADD_F64", "TRANS_F64")},
        "other_insts_per_wave_segment": {k: ws(classes.get(k, 0)) for k in VALU_COST if not k.endswith("F64")},
        "unclassified_valu_per_wave_segment": ws(other),
        "wave_cycle_split": {
            "active_inst_any": per.get("SQ_ACTIVE_INST_ANY", 0) / cyc,
            "wait_inst_any (issue stall)": per.get("SQ_WAIT_INST_ANY", 0) / cyc,
            "wait_any (waitcnt)": per.get("SQ_WAIT_ANY", 0) / cyc,
        },
        # (i) class-weighted VALU issue cycles of one SIMD per traversal
        "valu_class_cycles_per_segment": cycles / 64 / wave_segments if (wave_segments and complete) else None,
        "valu_class_complete": complete,
        # (ii) fp64 / fp32 FLOPs per traversal issued (64 lanes per instruction)
        "fp64_flops_per_segment": flops64 / seg_per_launch if (flops64 is not None and seg_per_launch) else None,
        "fp32_flops_per_segment": flops32 / seg_per_launch if (flops32 is not None and seg_per_launch) else None,
        "valu_lane_util": per["SQ_THREAD_CYCLES_VALU"] / (64 * act)
        if per.get("SQ_THREAD_CYCLES_VALU") and act else None,
        # diagnostic only (sum over co-resident waves, can pass 1)
        "valu_active_wave_sum": (4 * act / 1024) / (gui / 8) if (gui and act) else None,
        "clock_ghz_x_ms": (gui or 0) / 8 / 1e6,
        "waves_per_launch": per.get("SQ_WAVES"),
    }


def fold(out: str, dirs):
    lines = [bench_line(Path(str(d) + ".log")) for d in dirs]
    roofs = [ln["roofline"] for ln in lines]
    kernel, build = roofs[0]["kernel"], roofs[0]["build_id"]
    cfg = lines[0]["config"]

    class _A:  # pmc_key(args) wants scene / nx / ny / depth / bvh / precision
        scene, nx, ny, depth, bvh = cfg["scene"], cfg["nx"], cfg["ny"], cfg["max_depth"], cfg["bvh"]
        precision = cfg.get("precision", "fp64")

    key = pmc_key(_A)
    for r, ln in zip(roofs, lines):
        if r["kernel"] != kernel or r["build_id"] != build or ln["config"]["scene"] != cfg["scene"]:
            raise SystemExit("passes measured different kernels / builds / workloads")
    seg_per_launch = sum(r["segments_per_launch"] for r in roofs) / len(roofs)
    tot = defaultdict(float)
    disp = defaultdict(set)
    for d in dirs:
        for row in csv.DictReader(open(d / "run_counter_collection.csv")):
            if kernel not in row["Kernel_Name"]:  # e.g. "...::k_persist_sort<112, 8, true>(...)"
                continue
            tot[row["Counter_Name"]] += float(row["Counter_Value"])
            disp[row["Counter_Name"]].add((str(d), row["Dispatch_Id"]))
    per = {k: v / max(1, len(disp[k])) for k, v in tot.items()}  # per launch
    res = {
        "kernel": kernel,
        "build_id": build,
        "workload": key,
        "bench_workload": cfg["workload"],
        "source": "rocprofv3 --kernel-trace --pmc, one pass per counter group (scripts/pmc_passes.sh)",
        "launches_per_pass": max((len(v) for v in disp.values()), default=0),
        "segments_per_launch": seg_per_launch,
        "avg_launch_ms": sum(r["avg_launch_ms"] for r in roofs) / len(roofs),
        **derive(per, seg_per_launch),
        "raw_per_launch": per,
    }
    Path(out).parent.mkdir(parents=True, exist_ok=True)
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: res[k] for k in ("kernel", "build_id", "workload", "hbm_bytes_per_launch",
                                          "valu_insts_per_wave_segment", "valu_class_cycles_per_segment",
                                          "fp64_flops_per_segment", "valu_lane_util", "wave_cycle_split")}))


def refresh(paths):
    for p in paths:
        rec = json.loads(Path(p).read_text())
        for stale in ("valu_busy", "valu_busy_cycles_per_segment", "f32_insts_per_wave_segment"):
            rec.pop(stale, None)
        raw = rec.pop("raw_per_launch")
        rec.update(derive(raw, rec["segments_per_launch"]))
        rec["raw_per_launch"] = raw
        Path(p).write_text(json.dumps(rec, indent=1) + "\n")


if __name__ == "__main__":
    if sys.argv[1] == "--refresh":
        refresh(sys.argv[2:])
    else:
        fold(sys.argv[1], [Path(d) for d in sys.argv[2:]])
