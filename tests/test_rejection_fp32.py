"""The rejection loops decided in fp32 (rtw_device.h random_in_unit_sphere /
camera_ray, RTW_RIUS_FP32 / RTW_DISK_FP32): the fp32 value formed from a
canonical draw's second raw minstd output, fma((float)(raw - 1), fl32(2 / R),
-1), stays within 2^-21.5 of the fp64 2 x - 1 the reference forms from both
raw outputs, so |d32 - d| < 2^-18 for d = |p|^2 of three (or two) such
coordinates, and the loop's accept / reject bands (d32 < 1 - 2^-14, d32 >=
1 + 2^-14) decide as the fp64 test does.  Checked on the CPU with the device's
operations emulated exactly (an fp32 fma is the fp64 result of exact
operands rounded once), over random and edge raw draws."""
import numpy as np

R = 2147483646.0          # generate_canonical's R = 2^31 - 2 (rtw_device.h kCanonR)
DIV = 4611686009837453312.0  # (double)(R * R)
ONE_MINUS_ULP = np.nextafter(1.0, 0.0)


def canon(r1, r2):
    """libstdc++ generate_canonical<double, 53> of two raw draws (canon_raw)."""
    e1 = (r1 - 1).astype(np.float64)
    e2 = (r2 - 1).astype(np.float64)
    s = (0.0 + e1 * 1.0) + e2 * R
    v = s / DIV
    return np.where(v >= 1.0, ONE_MINUS_ULP, v)


def lead(r2):
    k2rf = np.float32(2.0 / R)
    e = (r2 - 1).astype(np.float32)
    return (e.astype(np.float64) * np.float64(k2rf) - 1.0).astype(np.float32)  # one rounding: an fp32 fma


def fma32(a, b, c):
    return (a.astype(np.float64) * b.astype(np.float64) + c.astype(np.float64)).astype(np.float32)


def raws(rng, n):
    r = rng.integers(1, 2**31 - 1, size=n, dtype=np.int64)
    edge = np.array([1, 2, 3, 2**31 - 2, 2**31 - 3, 2**30, 2**30 + 1, 2**30 - 1, 1073741823, 1073741824], np.int64)
    r[: edge.size] = edge
    return r


def test_lead_term_bound_and_decisions():
    rng = np.random.default_rng(7)
    n = 2_000_000
    z1, z2, y1, y2, x1, x2 = (raws(rng, n) for _ in range(6))
    for a in (z1, y1, x1):
        rng.shuffle(a)
    px, py, pz = (canon(a, b) * 2.0 - 1.0 for a, b in ((x1, x2), (y1, y2), (z1, z2)))
    fx, fy, fz = lead(x2), lead(y2), lead(z2)
    for f, p in ((fx, px), (fy, py), (fz, pz)):
        assert np.max(np.abs(f.astype(np.float64) - p)) < 2.0**-21.5
    # unit sphere: d = x^2 + y^2 + z^2 (no contraction), d32 = fma(x, x, fma(y, y, z * z))
    d = (px * px + py * py) + pz * pz
    d32 = fma32(fx, fx, fma32(fy, fy, (fz * fz).astype(np.float32)))
    assert np.max(np.abs(d32.astype(np.float64) - d)) < 2.0**-18
    acc = d32 < np.float32(1.0 - 2.0**-14)
    rej = ~(d32 < np.float32(1.0 + 2.0**-14))
    assert np.all(d[acc] < 1.0) and np.all(d[rej] >= 1.0)
    assert acc.mean() > 0.5 and (acc | rej).mean() > 0.9999
    # camera disk: d = x^2 + y^2 + 0, d32 = fma(x, x, y * y)
    d2 = (px * px + py * py) + 0.0 * 0.0
    d2_32 = fma32(fx, fx, (fy * fy).astype(np.float32))
    assert np.max(np.abs(d2_32.astype(np.float64) - d2)) < 2.0**-18
    acc2 = d2_32 < np.float32(1.0 - 2.0**-14)
    rej2 = ~(d2_32 < np.float32(1.0 + 2.0**-14))
    assert np.all(d2[acc2] < 1.0) and np.all(d2[rej2] >= 1.0)


def test_two_step_jumps_are_the_engine():
    """RTW_RNG_JUMP (rtw_device.h mr_jump): x -> (48271^2 mod m) x mod m with
    the Mersenne fold equals two minstd_rand steps, and the odd draw of a
    pair is 48271 x of the state before it -- on random and edge states; the
    fold's sum stays below 2m, so one conditional subtract completes it."""
    m = 2**31 - 1
    a = 48271
    a2 = 182605794
    assert a2 == a * a % m

    def fold(p):  # the device's mr_jump / mr_next on a product below 2^62
        r = (p & 0x7FFFFFFF) + (p >> 31)
        assert r < 2 * m
        return r - m if r >= m else r

    rng = np.random.default_rng(5)
    states = [1, 2, m - 1, m - 2, 2**30, 48271, a2] + [int(v) for v in rng.integers(1, m, size=20000)]
    for s in states:
        one = s * a % m
        two = one * a % m
        assert fold(s * a2) == two and fold(s * a) == one
