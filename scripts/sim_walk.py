"""Divergence model of the Book-2 (C5) group-BVH walks, on the CPU.

Traces paths with the oracle (rtw_oracle_trace: every segment's ray and hit
distance), then walks the ground-box and sphere-cluster group BVHs of the
flattened scene for each segment (fp64 slab tests, nearest child first,
closest distance shrinking as leaves are tested) and counts per segment the
nodes popped and the leaf items tested.  Segments are dealt into 64-lane
waves at random (the persistent kernel's lanes hold unrelated paths), and
a wave's while-while cost is modelled as the max over its lanes of the
counts: walked one group after the other (today: max(ground) + max(cluster))
or as one walk over both (max(ground + cluster)).

  python scripts/sim_walk.py [paths] [seed]
A measurement tool, not part of the product.
"""
import ctypes as C
import math
import random
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

from oracle_lib import oracle  # noqa: E402
from raytracingweekend_amd import _abi  # noqa: E402
from raytracingweekend_amd.render import SceneDesc  # noqa: E402


def slab(n, o, inv, t0, t1):
    for a in range(3):
        ta = (n.bmin[a] - o[a]) * inv[a]
        tb = (n.bmax[a] - o[a]) * inv[a]
        if ta > tb:
            ta, tb = tb, ta
        if ta != ta or tb != tb:
            continue
        t0 = max(t0, ta)
        t1 = min(t1, tb)
        if t1 < t0:
            return None
    return t0


def sphere_t(p, o, d, t_min, t_max):
    c = (p.p[0], p.p[1], p.p[2])
    r = p.p[3]
    oc = [o[k] - c[k] for k in range(3)]
    a = sum(x * x for x in d)
    b = sum(oc[k] * d[k] for k in range(3))
    cc = sum(x * x for x in oc) - r * r
    disc = b * b - a * cc
    if disc <= 0:
        return None
    sq = math.sqrt(disc)
    for t in ((-b - sq) / a, (-b + sq) / a):
        if t_min < t < t_max:
            return t
    return None


def box_t(desc, first, o, d, t_min, t_max):
    best = None
    for k in range(first, first + 6):
        q = desc.prims[k]
        K, A, B = {2: (2, 0, 1), 3: (1, 0, 2), 4: (0, 1, 2)}[q.type]
        if d[K] == 0:
            continue
        t = (q.p[4] - o[K]) / d[K]
        if t < t_min or t > (best if best is not None else t_max):
            continue
        a = o[A] + t * d[A]
        b = o[B] + t * d[B]
        if q.p[0] <= a <= q.p[1] and q.p[2] <= b <= q.p[3]:
            best = t
    return best


def walk(desc, root, o, d, t_max):
    inv = [1.0 / x if x != 0 else math.copysign(math.inf, x) for x in d]
    pops = items = 0
    stack = [root]
    while stack:
        n = desc.bvh_nodes[stack.pop()]
        pops += 1
        if slab(n, o, inv, 0.001, t_max) is None:
            continue
        if n.count > 0:
            for k in range(n.left, n.left + n.count):
                it = desc.bvh_items[k]
                items += 1
                if it & _abi.RTW_ITEM_BOX:
                    t = box_t(desc, it & _abi.RTW_ITEM_INDEX, o, d, 0.001, t_max)
                else:
                    t = sphere_t(desc.prims[it], o, d, 0.001, t_max)
                if t is not None and t < t_max:
                    t_max = t
            continue
        L, R = desc.bvh_nodes[n.left], desc.bvh_nodes[n.right]
        tl, tr = slab(L, o, inv, 0.001, t_max), slab(R, o, inv, 0.001, t_max)
        order = [(tl, n.left), (tr, n.right)]
        order = [x for x in order if x[0] is not None]
        order.sort(key=lambda x: -x[0])  # nearer pushed last
        stack.extend(i for _, i in order)
    return pops, items


def to_local(e, o, d):
    o, d = list(o), list(d)
    for k in range(e.n_ops):
        op, p = e.op[k], e.op_param[k]
        if op == _abi.RTW_OP_TRANSLATE:
            o = [o[a] - p[a] for a in range(3)]
        elif op == _abi.RTW_OP_ROTATE_Y:
            s, c = p[0], p[1]
            o = [c * o[0] - s * o[2], o[1], s * o[0] + c * o[2]]
            d = [c * d[0] - s * d[2], d[1], s * d[0] + c * d[2]]
    return o, d


def main():
    paths = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
    rnd = random.Random(int(sys.argv[2]) if len(sys.argv) > 2 else 1)
    flat = SceneDesc("book2_final", 1.0)
    tree = SceneDesc("book2_final", 1.0, use_bvh=True)
    d = tree.desc.contents if hasattr(tree.desc, "contents") else tree.desc
    groups = [(e, d.entries[e]) for e in range(d.n_entries) if d.entries[e].bvh_root >= 0]
    L = oracle()
    segs = []
    rows = (C.c_double * (8 * 64))()
    rad = (C.c_double * 3)()
    for k in range(paths):
        i, j = rnd.randrange(1600), rnd.randrange(1600)
        n = L.rtw_oracle_trace(C.byref(flat.desc if not hasattr(flat.desc, "contents") else flat.desc.contents),
                               C.byref(flat.camera), 1600, 1600, i, j, k, 50, 0, rad, rows, 64)
        for s in range(n):
            r = rows[8 * s:8 * s + 8]
            segs.append(((r[0], r[1], r[2]), (r[3], r[4], r[5]), r[6]))
    per = []
    for o, dd, t in segs:
        tm = t if t > 0 else 1e300
        counts = []
        for _, e in groups:
            lo, ld_ = to_local(e, o, dd)
            counts.append(walk(d, e.bvh_root, lo, ld_, tm))
        per.append(counts)
    rnd.shuffle(per)
    sep = uni = mean = 0.0
    waves = len(per) // 64
    for w in range(waves):
        lanes = per[64 * w:64 * w + 64]
        for g in range(len(groups)):
            sep += max(x[g][0] for x in lanes) + max(x[g][1] for x in lanes)
        uni += max(sum(x[g][0] for g in range(len(groups))) for x in lanes) + \
            max(sum(x[g][1] for g in range(len(groups))) for x in lanes)
        mean += sum(sum(x[g][0] + x[g][1] for g in range(len(groups))) for x in lanes) / 64
    # regrouped: blocks of 256 lanes sorted by which groups they walk past the root
    srt = 0.0
    blocks = len(per) // 256
    for b in range(blocks):
        lanes = per[256 * b:256 * b + 256]
        lanes = sorted(lanes, key=lambda x: tuple(x[g][0] > 1 for g in range(len(groups))))
        for w in range(4):
            wl = lanes[64 * w:64 * w + 64]
            for g in range(len(groups)):
                srt += max(x[g][0] for x in wl) + max(x[g][1] for x in wl)
    print(f"per wave, blocks of 256 sorted by the groups a lane walks: {srt / (4 * blocks):.1f}")
    print(f"segments {len(per)} waves {waves} groups {[e for e, _ in groups]}")
    for g, (ei, _) in enumerate(groups):
        p = [x[g][0] for x in per]
        it = [x[g][1] for x in per]
        print(f"  group entry {ei}: pops mean {sum(p) / len(p):.1f} max {max(p)}; items mean {sum(it) / len(it):.1f}"
              f" max {max(it)}; lanes walking past the root {sum(1 for v in p if v > 1) / len(p):.2f}")
    print(f"per wave: separate walks {sep / waves:.1f}, one walk {uni / waves:.1f}, lane mean {mean / waves:.1f}"
          f" -> lane utilisation {mean / sep:.2f} (separate) vs {mean / uni:.2f} (one walk)")


if __name__ == "__main__":
    main()
