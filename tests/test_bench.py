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

    # the roofline: VALU-bound with the record, HBM-only without
    monkeypatch.setattr(bench, "PMC_DIR", tmp_path)
    monkeypatch.setattr(bench.find_pmc, "__defaults__", (tmp_path,))
    r = bench.roofline(a, rec["kernel"], "abc", seg=2e9, ms=100.0, launches=2, algo=68 * 2e9)
    assert r["bound"] == "valu" and r["traffic"] == 1e9
    assert abs(r["achieved"] - 1000.0 * 1e9 / 64 / 0.05 / 1e9) < 1e-6 and r["unit"] == "G wave-instr/s"
    # a record with measured busy cycles and lane utilisation: the measured form
    rec2 = dict(rec, valu_busy_cycles_per_segment=50.0, valu_lane_util=0.5)
    (tmp_path / "T.json").write_text(json.dumps(rec2))
    r3 = bench.roofline(a, rec["kernel"], "abc", seg=2e9, ms=100.0, launches=2, algo=68 * 2e9)
    assert r3["unit"] == "G SIMD-cycles/s" and r3["peak"] == 1024 * 2.4
    assert abs(r3["achieved"] - 50.0 * 1e9 / 0.05 / 1e9) < 1e-6
    assert abs(r3["frac"] - round(1000.0 / 2457.6, 4)) < 1e-9 and r3["valu_lane_util"] == 0.5
    assert abs(r3["valu_useful_frac"] - round(1000.0 / 2457.6 * 0.5, 4)) < 1e-9
    assert abs(r3["issue_model"]["achieved"] - 1000.0 * 1e9 / 64 / 0.05 / 1e9) < 1e-6
    assert r["hbm"]["achieved"] == round(68 * 2e9 / 0.1 / 1e9, 2)
    r2 = bench.roofline(a, rec["kernel"], "stale", seg=2e9, ms=100.0, launches=2, algo=68 * 2e9)
    assert r2["bound"] == "hbm" and r2["traffic"] is None and "no PMC record" in r2["pmc"]


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
