"""bench.py's host logic on the CPU: the workloads are BASELINE.json's configs,
overrides make a run "custom", and a PMC record is attached only to the
kernel, build and workload it was taken on."""
import json
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


@pytest.fixture()
def bench(monkeypatch):
    monkeypatch.syspath_prepend(str(ROOT))
    import importlib
    import bench as b
    return importlib.reload(b)


def parse(bench, monkeypatch, *argv):
    monkeypatch.setattr(sys, "argv", ["bench.py", *argv])
    return bench.parse()


def test_workloads_are_the_baseline_configs(bench, monkeypatch):
    cfgs = json.loads((ROOT / "BASELINE.json").read_text())["configs"]
    w = bench.WORKLOADS
    assert (w["C2"]["nx"], w["C2"]["ny"], w["C2"]["spp"], w["C2"]["bvh"]) == (1200, 800, 256, False)
    assert "1200×800×256spp" in cfgs[1]
    assert (w["C3"]["spp"], w["C3"]["bvh"]) == (1024, True) and "1200×800×1024spp" in cfgs[2]
    assert (w["C4"]["nx"], w["C4"]["spp"]) == (800, 4096) and "800×800×4096spp" in cfgs[3]
    assert (w["C5"]["nx"], w["C5"]["spp"]) == (1600, 4096) and "1600×1600×4096spp" in cfgs[4]
    a = parse(bench, monkeypatch)
    assert (a.workload_key, a.scene, a.nx, a.ny, a.spp, a.depth, a.bvh) == ("T", "cornell_box", 800, 800, 1024, 50,
                                                                           False)
    assert a.scaling == "strong"
    c = parse(bench, monkeypatch, "--workload", "C3")
    assert (c.scene, c.bvh, c.spp) == ("random_balls", True, 1024) and c.workload_key == "C3"
    d = parse(bench, monkeypatch, "--spp", "64")
    assert d.workload_key == "custom" and d.spp == 64 and "custom" in d.label
    e = parse(bench, monkeypatch, "--spp", "1024")  # same as the workload: not custom
    assert e.workload_key == "T"


def test_pmc_record_must_match_kernel_build_and_workload(bench, monkeypatch, tmp_path):
    rec = {"kernel": "k_persist_sort<112, 8, true>", "build_id": "abc", "workload": "cornell_box 800x800 depth 50",
           "segments_per_launch": 1e9, "hbm_bytes_per_launch": 1e9, "valu_insts_per_wave_segment": 1000.0}
    (tmp_path / "T.json").write_text(json.dumps(rec))
    got, src = bench.find_pmc(rec["kernel"], "abc", rec["workload"], tmp_path)
    assert got == rec and src == "T.json"
    assert bench.find_pmc(rec["kernel"], "other-build", rec["workload"], tmp_path)[0] is None
    assert bench.find_pmc("k_persist<2, 12, false, true>", "abc", rec["workload"], tmp_path)[0] is None
    assert bench.find_pmc(rec["kernel"], "abc", "cornell_box 400x400 depth 50", tmp_path)[0] is None
    a = parse(bench, monkeypatch)
    assert bench.pmc_key(a) == "cornell_box 800x800 depth 50"

    # the roofline: the 8(d) HBM headline always; with the record its traffic
    # and the bounded VALU figures beside it
    monkeypatch.setattr(bench, "PMC_DIR", tmp_path)
    monkeypatch.setattr(bench.find_pmc, "__defaults__", (tmp_path,))
    r = bench.roofline(a, rec["kernel"], "abc", seg=2e9, ms=100.0, launches=2, algo=68 * 2e9)
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["traffic"] == 1e9
    assert r["achieved"] == round(68 * 2e9 / 0.1 / 1e9, 2) and r["frac"] == round(r["achieved"] / 8000.0, 4)
    assert "class_weighted" not in r["valu"]  # the record holds no instruction classes
    # a record with class-weighted cycles, FLOPs and lane utilisation
    rec2 = dict(rec, valu_class_cycles_per_segment=50.0, valu_lane_util=0.5, fp64_flops_per_segment=400.0,
                write_bytes_per_launch=5e8)
    (tmp_path / "T.json").write_text(json.dumps(rec2))
    r3 = bench.roofline(a, rec["kernel"], "abc", seg=2e9, ms=100.0, launches=2, algo=68 * 2e9)
    cw = r3["valu"]["class_weighted"]
    assert cw["unit"] == "G SIMD-cycles/s" and cw["peak"] == 1024 * 2.4
    assert abs(cw["achieved"] - 50.0 * 1e9 / 0.05 / 1e9) < 1e-6
    assert abs(cw["frac"] - round(1000.0 / 2457.6, 4)) < 1e-9 and r3["valu"]["lane_util"] == 0.5
    assert abs(r3["valu"]["useful_frac"] - round(1000.0 / 2457.6 * 0.5, 4)) < 1e-9
    fl = r3["valu"]["fp64_flops"]
    assert abs(fl["issued"] - 400.0 * 1e9 / 0.05 / 1e12) < 1e-9 and fl["peak"] == 78.6
    assert abs(fl["achieved"] - 0.5 * 400.0 * 1e9 / 0.05 / 1e12) < 1e-9
    assert r3["write_bytes"] == 5e8
    assert "pmc_clock_ghz" not in r3  # the record carries no clock
    rec5 = dict(rec2, clock_ghz_x_ms=237.0, avg_launch_ms=100.0)  # GRBM cycles: 2.37 GHz
    (tmp_path / "T.json").write_text(json.dumps(rec5))
    r5 = bench.roofline(a, rec["kernel"], "abc", seg=2e9, ms=100.0, launches=2, algo=68 * 2e9)
    assert r5["pmc_clock_ghz"] == 2.37
    r2 = bench.roofline(a, rec["kernel"], "stale", seg=2e9, ms=100.0, launches=2, algo=68 * 2e9)
    assert r2["bound"] == "hbm" and r2["traffic"] is None and "no PMC record" in r2["pmc"] and "valu" not in r2
    # a fraction above 1 is refused, never reported
    rec4 = dict(rec2, valu_class_cycles_per_segment=5000.0)
    (tmp_path / "T.json").write_text(json.dumps(rec4))
    with pytest.raises(ValueError, match="not a roofline fraction"):
        bench.roofline(a, rec["kernel"], "abc", seg=2e9, ms=100.0, launches=2, algo=68 * 2e9)


def test_pmc_derivation_is_bounded(monkeypatch):
    """scripts/pmc_to_json.derive: class-weighted cycles from the instruction
    classes (unclassified VALU at the cheapest rate), FLOPs per traversal; a
    record missing a class gives no class-weighted figure."""
    monkeypatch.syspath_prepend(str(ROOT / "scripts"))
    import importlib
    import bench as b
    import pmc_to_json as p
    importlib.reload(p)
    per = {"SQ_INSTS_VALU": 1000.0, "SQ_ACTIVE_INST_VALU": 100.0, "SQ_THREAD_CYCLES_VALU": 3200.0,
           "SQ_INSTS_VALU_FLOPS_FP64": 6400.0, "SQ_INSTS_VALU_FLOPS_FP64_TRANS": 64.0,
           "FETCH_SIZE": 1.0, "WRITE_SIZE": 2.0}
    per.update({f"SQ_INSTS_VALU_{k}": 50.0 for k in b.VALU_COST})
    d = p.derive(per, 640.0)  # 10 wave-segments
    other = 1000.0 - 50.0 * len(b.VALU_COST)
    want = (sum(50.0 * c for c in b.VALU_COST.values()) + b.VALU_COST_OTHER * other) / 64 / 10
    assert abs(d["valu_class_cycles_per_segment"] - want) < 1e-9
    assert d["fp64_flops_per_segment"] == 6400.0 * 64 / 640.0 and d["valu_lane_util"] == 0.5
    assert d["hbm_bytes_per_launch"] == 2048 + 2048
    del per["SQ_INSTS_VALU_CVT"]
    assert p.derive(per, 640.0)["valu_class_cycles_per_segment"] is None


def test_committed_records_stay_below_peak(bench):
    """Every committed PMC record, priced at its own launch time, gives
    class-weighted VALU and fp64 FLOP fractions of at most 1."""
    d = ROOT / "profiles" / "pmc"
    for f in sorted(d.glob("*.json")) if d.is_dir() else []:
        p = json.loads(f.read_text())
        ms = p.get("avg_launch_ms")
        if not ms:
            continue
        secs = ms * 1e-3
        if p.get("valu_class_cycles_per_segment"):
            assert p["valu_class_cycles_per_segment"] * p["segments_per_launch"] / secs / 1e9 <= bench.VALU_SIMD_GCYC, f.name
        if p.get("fp64_flops_per_segment"):
            assert p["fp64_flops_per_segment"] * p["segments_per_launch"] / secs / 1e12 <= bench.FP64_PEAK_TFLOPS, f.name


def test_committed_pmc_records_are_complete():
    """Every committed record names its kernel, build and workload."""
    d = ROOT / "profiles" / "pmc"
    for f in sorted(d.glob("*.json")) if d.is_dir() else []:
        p = json.loads(f.read_text())
        for k in ("kernel", "build_id", "workload", "segments_per_launch", "hbm_bytes_per_launch",
                  "valu_insts_per_wave_segment"):
            assert p.get(k) is not None, f"{f.name}: {k}"


def test_spawn_starts_one_rank_per_gpu(bench, monkeypatch):
    """--gpus N started directly: bench.py runs torch.distributed.run as a
    child (never exec) with N ranks on 127.0.0.1 and the same arguments, and
    exits with its status."""
    calls = []

    def fake_call(cmd, env=None):
        calls.append((cmd, env))
        return 7

    monkeypatch.setattr(bench.subprocess, "call", fake_call)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "2", "--workload", "C4"])
    a = bench.parse()
    assert bench.spawn(a) == 7
    (cmd, env), = calls
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nnodes=1" in cmd and "--nproc-per-node=4" in cmd and "--master-addr=127.0.0.1" in cmd
    port = [c for c in cmd if c.startswith("--master-port=")]
    assert len(port) == 1 and 0 < int(port[0].split("=")[1]) < 65536
    i = cmd.index(str((ROOT / "bench.py").resolve()))
    assert cmd[i + 1:] == ["--gpus", "4", "--steps", "2", "--workload", "C4"]
    assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"

    # main() spawns (and exits with the child's status) only outside torch.distributed.run
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    with pytest.raises(SystemExit) as ex:
        bench.main()
    assert ex.value.code == 7 and len(calls) == 2


def test_cpu_baseline_sample_is_bounded(bench, monkeypatch):
    """The CPU baseline renders a bounded sample: every stride-th row at a
    few spp, sized per scene."""
    for scene, (spp, stride) in bench.CPU_SAMPLE.items():
        nx, ny = {"cornell_box": (800, 800), "random_balls": (1200, 800), "book2_final": (1600, 1600)}[scene]
        samples = nx * len(range(0, ny, stride)) * spp
        assert samples <= 25_000_000, scene


def test_cpu_baseline_port_is_one_threaded_call(bench, monkeypatch, built):
    """Without oracle/_ref/rtw_ref the C restatement is timed in ONE call over
    the strided rows with every requested thread (it was one call
    per row), and the strided call renders exactly the rows one-row calls do."""
    import numpy as np
    monkeypatch.syspath_prepend(str(ROOT / "tests"))
    import oracle_lib
    from raytracingweekend_amd.render import SceneDesc
    calls = []
    real = oracle_lib.oracle_sums

    def spy(*a, **k):
        calls.append(k)
        return real(*a, **k)
    monkeypatch.setattr(oracle_lib, "oracle_sums", spy)
    a = parse(bench, monkeypatch, "--scene", "cornell_box", "--nx", "32", "--ny", "24", "--cpu-spp", "2")
    out = bench.cpu_baseline(a, 4, use_reference=False)
    assert out["kind"] == "port" and out["cores"] == 4 and out["value"] > 0
    assert len(calls) == 1 and calls[0]["threads"] == 4 and calls[0]["rows"] == (0, 24, 1)

    sd = SceneDesc("random_balls", 1.5, False)
    strided, seg = real(sd, 24, 16, 2, 10, 3, threads=4, rows=(1, 4, 4))
    rowwise = np.zeros_like(strided)
    segs = 0
    for j in (1, 5, 9, 13):
        r, s = real(sd, 24, 16, 2, 10, 3, threads=1, rows=(j, 1))
        rowwise += r
        segs += s
    assert seg == segs and np.array_equal(strided, rowwise)


def test_bench_line_drops_an_unbounded_valu_figure(bench):
    """In the bench line a VALU fraction above 1 (a slightly stale PMC
    record) is dropped with a warning instead of aborting the run before the
    line is printed; roofline() itself keeps refusing it."""
    out = {"frac": 0.2, "valu": {"class_weighted": {"frac": 1.3}}}
    got = bench.bounded_valu(out)
    assert "valu" not in got and "not a roofline fraction" in got["warning"] and got["frac"] == 0.2
    ok = {"frac": 0.2, "valu": {"class_weighted": {"frac": 0.7}}}
    assert bench.bounded_valu(dict(ok)) == ok


def test_shared_gpu_rehearsal_is_named_in_the_line(bench, monkeypatch):
    """RTW_BENCH_SHARED_GPU=1 (every rank on cuda:0, gloo collectives: the
    one-GPU rehearsal of the N > 1 path, tests/test_gpu_multirank.py) must
    never pass for an RCCL line: config.parallelism says which it was."""
    a = parse(bench, monkeypatch, "--gpus", "2")
    phases = bench.rank_phases({}, 1)
    samples = a.nx * a.ny * a.spp * a.steps
    line = bench.result_line(a, 2, a.spp, 1.0, samples, 0, 0.0, None, phases)
    assert line["config"]["parallelism"] == "spp-shard x2 + RCCL reduce"
    a.shared_gpu = True
    line = bench.result_line(a, 2, a.spp, 1.0, samples, 0, 0.0, None, phases)
    assert "gloo" in line["config"]["parallelism"] and "rehearsal" in line["config"]["parallelism"]
    assert "RCCL" not in line["config"]["parallelism"]
