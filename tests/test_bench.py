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
    assert abs(r["achieved"] - 1000.0 * 1e9 / 64 / 0.05 / 1e9) < 1e-6
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
