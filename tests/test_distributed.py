"""N > 1 path on CPU: world_size-2 gloo ranks run bench.py's step
(raytracingweekend_amd.distributed.render_step) with the oracle standing in
for each rank's GPU renderer and numpy for the device finalize (test-only
injection); the reduced canvas on rank 0 equals the single-process render."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from raytracingweekend_amd.distributed import render_sharded, render_step, sample_range

NX, NY, SPP, DEPTH, SEED = 20, 16, 5, 50, 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _oracle_fn(sd):
    from oracle_lib import oracle_sums

    def fn(spp_begin, spp_count, row_begin, row_step, accum):
        rows = list(range(row_begin, NY, row_step))
        out = np.zeros(NX * NY * 3)
        for j in rows:
            s, _ = oracle_sums(sd, NX, NY, SPP, DEPTH, SEED, threads=1, rows=(j, 1), spp_begin=spp_begin,
                               spp_count=spp_count)
            out += s
        accum += torch.from_numpy(out)

    return fn


def _worker(rank, world, port, mode, q):
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    sys.path.insert(0, str(root))
    sys.path.insert(0, str(root / "tests"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from raytracingweekend_amd.render import SceneDesc
    sd = SceneDesc("cornell_box", NX / NY)
    accum = torch.zeros(NX * NY * 3, dtype=torch.float64)
    if mode == "phases":
        # bench.py's timed step: render_step's per-rank phase times, reduced
        # over the ranks by bench.rank_phases and put into the rank-0 line
        import bench
        from oracle_lib import finalize_np
        canvas_t = torch.zeros(NX * NY * 3, dtype=torch.float64)
        ms = {}

        def fin(acc, canvas):
            canvas.copy_(torch.from_numpy(finalize_np(acc.numpy(), SPP)))

        fn = _oracle_fn(sd)
        stats = {"samples": 0}

        def counting(b, c, r0, rs, acc):
            fn(b, c, r0, rs, acc)
            stats["samples"] += NX * NY * c

        render_step(counting, fin, accum, canvas_t, NX, NY, SPP, timings=ms)
        local = dict(ms, kernel=10.0 * (rank + 1))  # a stand-in kernel time per rank
        phases = bench.rank_phases(local, world)
        # a stand-in device record per rank (no GPU here): bench.device_record's fields
        placement = bench.rank_devices(world, rank, rank, {"device": rank, "pci_bus_id": f"0000:{0x11 + rank:02x}:00",
                                                           "name": "stand-in", "arch": "gfx950"})
        t = torch.tensor([float(stats["samples"])], dtype=torch.float64)
        dist.all_reduce(t)
        if rank == 0:
            import sys as _s
            _s.argv = ["bench.py", "--gpus", "2", "--steps", "1", "--scene", "cornell_box", "--nx", str(NX),
                       "--ny", str(NY), "--spp", str(SPP)]
            a = bench.parse()
            line = bench.result_line(a, world, SPP, 0.5, float(t.item()), 1000.0, 1.0, None, phases, placement)
            q.put((line, ms))
        dist.destroy_process_group()
        return
    if mode == "step":
        # bench.py's step: render_step with a finalize into a canvas tensor
        from oracle_lib import finalize_np
        canvas_t = torch.full((NX * NY * 3,), -1.0, dtype=torch.float64)

        def fin(acc, canvas):
            canvas.copy_(torch.from_numpy(finalize_np(acc.numpy(), SPP)))

        for _ in range(2):  # a warmup step and a timed one: the accumulator restarts from zero
            render_step(_oracle_fn(sd), fin, accum, canvas_t, NX, NY, SPP)
        canvas = canvas_t.numpy() if rank == 0 else None
        if rank != 0:
            assert canvas_t[0] == -1.0  # only rank 0 finalises
    else:
        canvas = render_sharded(_oracle_fn(sd), NX, NY, SPP, accum, mode=mode)
    if rank == 0:
        q.put(canvas)
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["spp", "rows", "step"])
def test_two_rank_gloo_matches_single(built, mode):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, mode, q)) for r in range(2)]
    for p in procs:
        p.start()
    canvas = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    from oracle_lib import finalize_np, oracle_sums
    from raytracingweekend_amd.render import SceneDesc
    full, _ = oracle_sums(SceneDesc("cornell_box", NX / NY), NX, NY, SPP, DEPTH, SEED)
    want = finalize_np(full, SPP)
    if mode == "rows":
        assert np.array_equal(canvas, want)
    else:
        assert np.allclose(canvas, want, rtol=1e-13, atol=1e-13)


def test_sample_range_partition():
    for spp in (1, 7, 64, 1024):
        for world in (1, 2, 3, 8):
            got = [sample_range(spp, world, r) for r in range(world)]
            assert sum(c for _, c in got) == spp
            pos = 0
            for b, c in got:
                assert b == pos
                pos += c


def test_two_rank_line_carries_per_rank_phases(built):
    """bench.py --gpus N: the rank-0 JSON line carries each phase's max / min
    over the ranks and rank 0's value (all_reduce MAX / MIN, as the step time
    is) -- the diagnosis of a slow rank, the reduce and the finalize in the
    driver's N > 1 runs (round-4 verdict, next #8)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, "phases", q)) for r in range(2)]
    for p in procs:
        p.start()
    line, ms0 = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    ph = line["rank_phases_ms"]
    assert set(ph) == {"kernel", "render", "reduce", "finalize"}
    assert ph["kernel"] == {"max": 20.0, "min": 10.0, "rank0": 10.0}
    for k in ("render", "reduce", "finalize"):
        assert ph[k]["max"] >= ph[k]["rank0"] >= ph[k]["min"] >= 0.0, (k, ph[k])
        assert abs(ph[k]["rank0"] - round(ms0[k], 3)) < 1e-9, k
    assert ph["render"]["min"] > 0.0  # both ranks rendered their shard
    assert line["n_gpus"] == 2 and line["value"] == round(NX * NY * SPP / 0.5 / 1e6, 3)
    assert line["config"]["parallelism"] == "spp-shard x2 + RCCL reduce"
    # who ran where, gathered over the process group (round-5 verdict, next #5)
    assert line["process_group"] == {"backend": "gloo", "world_size": 2, "timeout_s": bench_timeout()}
    assert [r["rank"] for r in line["ranks"]] == [0, 1]
    assert [r["local_rank"] for r in line["ranks"]] == [0, 1]
    assert [r["pci_bus_id"] for r in line["ranks"]] == ["0000:11:00", "0000:12:00"]
    assert line["distinct_devices"] == 2


def bench_timeout():
    import bench
    return bench.PG_TIMEOUT_S


def test_one_rank_placement_without_a_group():
    import bench
    p = bench.rank_devices(1, 0, 0, {"device": 0, "pci_bus_id": "0000:05:00", "name": "x", "arch": "gfx950"})
    assert p["process_group"] == {"backend": None, "world_size": 1, "timeout_s": None}
    assert p["ranks"] == [{"rank": 0, "local_rank": 0, "device": 0, "pci_bus_id": "0000:05:00", "name": "x",
                           "arch": "gfx950"}]
    assert p["distinct_devices"] == 1
