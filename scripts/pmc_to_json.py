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

Usage: python scripts/pmc_to_json.py <out.json> <pass-dir> [<pass-dir> ...]
       (each pass dir = gpurun_out/pmc_<tag>_<i>, with pmc_<tag>_<i>.log beside it)
"""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from bench import pmc_key  # noqa: E402


def bench_line(log: Path) -> dict:
    for line in reversed(log.read_text().splitlines()):
        if line.startswith("{"):
            return json.loads(line)
    raise SystemExit(f"{log}: no bench line")


out, dirs = sys.argv[1], [Path(d) for d in sys.argv[2:]]
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
fetch = per.get("FETCH_SIZE", 0.0) * 1024 * 2
write = per.get("WRITE_SIZE", 0.0) * 1024
wave_segments = seg_per_launch / 64
res = {
    "kernel": kernel,
    "build_id": build,
    "workload": key,
    "bench_workload": cfg["workload"],
    "source": "rocprofv3 --kernel-trace --pmc, one pass per counter group (scripts/pmc_passes.sh)",
    "launches_per_pass": max((len(v) for v in disp.values()), default=0),
    "hbm_bytes_per_launch": fetch + write,
    "fetch_bytes_per_launch": fetch,
    "write_bytes_per_launch": write,
    "segments_per_launch": seg_per_launch,
    "valu_insts_per_wave_segment": per.get("SQ_INSTS_VALU", 0) / wave_segments if wave_segments else None,
    "salu_insts_per_wave_segment": per.get("SQ_INSTS_SALU", 0) / wave_segments if wave_segments else None,
    "f64_insts_per_wave_segment": {k[14:]: per.get(k, 0) / wave_segments for k in
                                   ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64",
                                    "SQ_INSTS_VALU_TRANS_F64")} if wave_segments else None,
    "wave_cycle_split": {
        "active_inst_any": per.get("SQ_ACTIVE_INST_ANY", 0) / max(1, per.get("SQ_WAVE_CYCLES", 1)),
        "wait_inst_any (issue stall)": per.get("SQ_WAIT_INST_ANY", 0) / max(1, per.get("SQ_WAVE_CYCLES", 1)),
        "wait_any (waitcnt)": per.get("SQ_WAIT_ANY", 0) / max(1, per.get("SQ_WAVE_CYCLES", 1)),
    },
    # measured VALU issue: SQ_ACTIVE_INST_VALU is in quad-cycles summed over
    # the SIMDs, GRBM_GUI_ACTIVE in cycles summed over the 8 XCDs
    "valu_busy_cycles_per_segment": 4 * per.get("SQ_ACTIVE_INST_VALU", 0) / seg_per_launch if seg_per_launch else None,
    "valu_busy": (4 * per.get("SQ_ACTIVE_INST_VALU", 0) / 1024) / (per["GRBM_GUI_ACTIVE"] / 8)
    if per.get("GRBM_GUI_ACTIVE") else None,
    "clock_ghz_x_ms": per.get("GRBM_GUI_ACTIVE", 0) / 8 / 1e6,
    # lanes doing work per VALU instruction cycle (rocprof's VALUUtilization):
    # the divergence measure the VALU fraction alone cannot show
    "valu_lane_util": per["SQ_THREAD_CYCLES_VALU"] / (64 * per["SQ_ACTIVE_INST_VALU"])
    if per.get("SQ_THREAD_CYCLES_VALU") and per.get("SQ_ACTIVE_INST_VALU") else None,
    "f32_insts_per_wave_segment": {k[14:]: per.get(k, 0) / wave_segments for k in
                                   ("SQ_INSTS_VALU_FMA_F32", "SQ_INSTS_VALU_ADD_F32", "SQ_INSTS_VALU_MUL_F32",
                                    "SQ_INSTS_VALU_TRANS_F32", "SQ_INSTS_VALU_CVT", "SQ_INSTS_VALU_INT32",
                                    "SQ_INSTS_VALU_INT64")} if wave_segments else None,
    "waves_per_launch": per.get("SQ_WAVES"),
    "raw_per_launch": per,
}
Path(out).parent.mkdir(parents=True, exist_ok=True)
json.dump(res, open(out, "w"), indent=1)
print(json.dumps({k: res[k] for k in ("kernel", "build_id", "workload", "hbm_bytes_per_launch",
                                      "valu_insts_per_wave_segment", "valu_busy", "valu_lane_util",
                                      "wave_cycle_split")}))
