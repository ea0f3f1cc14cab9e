"""The oracle pinned to the reference (CPU).

tests/golden/ was produced by the reference's own code (oracle/_ref/rtw_ref,
compiled from /root/reference by oracle/Makefile; generator
oracle/make_golden.py).  The C restatement must reproduce those renders BIT FOR
BIT from the scenes the product's host API builds — which pins the oracle, the
host scene API, the flattener and the RNG stream definition at once.
"""
import ctypes as C
import json
from pathlib import Path

import numpy as np
import pytest

from oracle_lib import finalize_np, oracle, oracle_sums

GOLD = Path(__file__).resolve().parent / "golden"
CASES = json.loads((GOLD / "renders.json").read_text())


@pytest.fixture(scope="module")
def api(built):
    from raytracingweekend_amd import render
    return render


@pytest.mark.parametrize("case", CASES, ids=[c["case"] for c in CASES])
def test_oracle_matches_reference_render(api, case):
    sd = api.SceneDesc(case["scene"], case["nx"] / case["ny"])
    sums, seg = oracle_sums(sd, case["nx"], case["ny"], case["spp"], case["max_depth"], seed=case["seed"])
    gold = np.load(GOLD / f"render_{case['case']}.npy")
    assert seg == case["segments"]
    assert np.array_equal(sums, gold), f"max diff {np.abs(sums - gold).max()}"


def test_oracle_threads_do_not_change_results(api):
    sd = api.SceneDesc("cornell_box", 1.0)
    a, _ = oracle_sums(sd, 24, 24, 3, 50, seed=4, threads=1)
    b, _ = oracle_sums(sd, 24, 24, 3, 50, seed=4, threads=4)
    assert np.array_equal(a, b)


def test_oracle_sample_ranges_compose(api):
    """Sample-range shards of the oracle sum to the full render (same order)."""
    sd = api.SceneDesc("cornell_box", 1.0)
    full, _ = oracle_sums(sd, 16, 16, 5, 50, seed=2)
    a, _ = oracle_sums(sd, 16, 16, 5, 50, seed=2, spp_begin=0, spp_count=3)
    b, _ = oracle_sums(sd, 16, 16, 5, 50, seed=2, spp_begin=3, spp_count=2)
    assert np.allclose(a + b, full, rtol=1e-13, atol=1e-13)


def _canonical_py(state):
    """libstdc++ generate_canonical<double,53>(std::minstd_rand) in Python."""
    R = 2147483646
    draws = []
    for _ in range(2):
        state = state * 48271 % 2147483647
        draws.append(state)
    tmp2 = float(R * R)  # (double)((long double)R * R): exact product, one rounding
    s = float(draws[0] - 1) + float(draws[1] - 1) * float(R)
    u = s / tmp2
    return (np.nextafter(1.0, 0.0) if u >= 1.0 else u), state


def test_canonical_matches_libstdcxx_definition(built):
    rng = np.random.default_rng(0)
    for st in [1, 2, 2147483646, 48271, *rng.integers(1, 2147483646, 200).tolist()]:
        s = C.c_uint32(int(st))
        u = oracle().rtw_oracle_canonical(C.byref(s))
        u2, st2 = _canonical_py(int(st))
        assert u == u2 and s.value == st2


def test_canonical_first_draws_of_default_engine(built):
    """minstd_rand's default state (1): the first raw draws are 48271 and
    182605794 (the C++ standard's 10000th-value check is 399268537)."""
    st = 1
    seq = []
    for _ in range(10000):
        st = st * 48271 % 2147483647
        seq.append(st)
    assert seq[0] == 48271 and seq[1] == 182605794 and seq[-1] == 399268537
    s = C.c_uint32(1)
    u = oracle().rtw_oracle_canonical(C.byref(s))
    assert u == (float(48271 - 1) + float(182605794 - 1) * 2147483646.0) / float(2147483646 * 2147483646)


def _splitmix64(x):
    M = (1 << 64) - 1
    z = (x + 0x9E3779B97F4A7C15) & M
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
    return z ^ (z >> 31)


def test_path_seed_definition(built):
    from raytracingweekend_amd import lib
    for seed, pixel, s in [(0, 0, 0), (7, 12345, 3), (2**63 + 5, 2**32 - 1, 2**31), (1, 639999, 1023)]:
        want = 1 + _splitmix64(_splitmix64(seed) ^ ((s << 32) ^ pixel)) % 2147483646
        assert lib().rtw_path_seed(seed, pixel, s) == want
        assert oracle().rtw_oracle_path_seed(seed, pixel, s) == want


def test_perlin_known_answers(api):
    gold = json.loads((GOLD / "perlin.json").read_text())
    sd = api.SceneDesc("light_sample", 2.0)  # uses noise_texture -> perlin tables
    d = sd.desc
    assert d.has_perlin == 1
    rv = np.ctypeslib.as_array(d.perlin_ranvec, shape=(768,)).reshape(256, 3)
    pm = np.ctypeslib.as_array(d.perlin_perm, shape=(768,)).reshape(3, 256)
    assert np.array_equal(rv, np.array(gold["ranvec"]))
    assert np.array_equal(pm[0], gold["perm_x"]) and np.array_equal(pm[1], gold["perm_y"])
    assert np.array_equal(pm[2], gold["perm_z"])
    assert np.array_equal(pm[0], pm[1]) and np.array_equal(pm[1], pm[2])
    for smp in gold["samples"]:
        p = (C.c_double * 3)(*smp["p"])
        assert oracle().rtw_oracle_noise(sd.ptr, C.byref(p)) == smp["noise"]
        assert oracle().rtw_oracle_turb(sd.ptr, C.byref(p)) == smp["turb"]


def test_finalize_matches_reference_rule(api):
    """RayTracingWeekend.cpp:241-244 (library) == numpy restatement, NaN kept."""
    rng = np.random.default_rng(1)
    acc = rng.random(16 * 8 * 3) * 300.0
    acc[5] = np.nan
    acc[7] = 0.0
    got = api.finalize(acc, 16, 8, 64)
    want = finalize_np(acc, 64)
    assert np.array_equal(np.isnan(got), np.isnan(want))
    m = ~np.isnan(want)
    assert np.array_equal(got[m], want[m])
