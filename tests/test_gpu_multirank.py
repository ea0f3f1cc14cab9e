"""The N > 1 bench path on a real GPU: bench.py --gpus 2 as two processes
(torch.distributed.run, started by bench.py itself), both rendering on cuda:0
with the collectives over gloo (RTW_BENCH_SHARED_GPU=1: RCCL refuses two
ranks on one device, and this pool's boxes have one GPU).  Everything but the
transport is the driver's 8-GPU run: per-rank sample shards through the
C-ABI renderer, the reduce of the fp64 sums to rank 0, the GPU finalize, the
max-over-ranks step time and the per-rank phase record.  The rank-0 canvas
equals a one-process render of the same image (the sharded sums differ from
one-process sums only in fp64 addition order: quantised 8-bit values agree).
"""
import json
import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
ARGS = ["--workload", "T", "--nx", "96", "--ny", "64", "--spp", "64", "--steps", "2", "--warmup", "1",
        "--no-cpu-baseline"]


def _bench(gpus, ppm, extra_env):
    env = {**os.environ, **extra_env}
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", str(gpus), *ARGS, "--ppm", str(ppm)],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    return json.loads(lines[0])


def _ppm(path):
    data = Path(path).read_text().split()
    assert data[0] == "P3"
    nx, ny = int(data[1]), int(data[2])
    return np.array(data[4:], dtype=np.int32).reshape(ny, nx, 3)


@pytest.mark.gpu
def test_two_ranks_on_one_gpu_match_one_rank(tmp_path):
    one = _bench(1, tmp_path / "one.ppm", {})
    two = _bench(2, tmp_path / "two.ppm", {"RTW_BENCH_SHARED_GPU": "1"})
    print(json.dumps(one))
    print(json.dumps(two))
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2
    assert "rehearsal" in two["config"]["parallelism"]
    assert two["config"]["spp_per_gpu"] == 32 and two["config"]["global_batch"] == 96 * 64 * 64
    ph = two["rank_phases_ms"]
    for k in ("kernel", "render", "reduce", "finalize"):
        assert ph[k]["max"] >= ph[k]["rank0"] >= ph[k]["min"] >= 0.0, (k, ph[k])
    assert ph["kernel"]["min"] > 0.0  # both ranks launched the traversal kernel
    # both lines counted the same traversals per sample (the same paths)
    assert two["segments_per_sample"] == one["segments_per_sample"]
    a, b = _ppm(tmp_path / "one.ppm"), _ppm(tmp_path / "two.ppm")
    assert a.shape == b.shape == (64, 96, 3)
    assert np.array_equal(a, b)
