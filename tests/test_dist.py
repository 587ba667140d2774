"""Multi-rank path on CPU: world_size 2 over gloo (127.0.0.1).

Each rank renders its shard (the oracle's fp32 kernel mirror stands in for
the per-GPU kernel here; the GPU tests cover kernel == mirror), rank 0
gathers, and the gathered frame must equal a single-rank render bit for bit
(strong: interleaved row tiles) or average to it (weak: sample stripes);
the bench's barrier + max-over-ranks timing reduction is exercised too."""
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parent.parent


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _render_rows(rows, w, h, spp, depth, sample_begin=0):
    import oracle
    from rtclj import raytracing as R
    sc = R.Scene.from_bodies(R.hittables)
    cam = R.camera(w, h, **R.REFERENCE_CAMERA)
    out = np.zeros((len(rows), w, 3), np.float32)
    for i, r in enumerate(rows):
        out[i] = oracle.render(oracle.MODE_MIRROR32, sc.sphere.astype(np.float64), sc.kind, sc.mat.astype(np.float64),
                               cam.as_list(), cam.defocus, w, h, spp, depth, rows=(r, r + 1),
                               sample_begin=sample_begin, nthreads=2)[0][0]
    return out


def _worker(rank, world, port, scaling, q):
    sys.path[:0] = [str(ROOT), str(ROOT / "raytracing-clj_amd")]
    import torch
    import torch.distributed as dist
    from rtclj.shard import shard_params, shard_rows
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    w, h, spp, depth = 40, 22, 4, 20
    p = shard_params(world, rank, w, h, spp, depth, scaling=scaling)
    rows = shard_rows(h, p.get("row_tile", 8), p.get("tile_first", 0), p.get("tile_step", 0))
    img = _render_rows(rows, w, h, spp, depth, p.get("sample_begin", 0))
    dist.barrier()
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)          # bench.py's max-over-ranks timing
    parts = [None] * world
    dist.all_gather_object(parts, (rows, img))
    if rank == 0:
        q.put((t.item(), parts))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("scaling", ["strong", "weak"])
def test_two_rank_gloo_shards(scaling):
    from rtclj.shard import gather_rows
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, scaling, q)) for r in range(world)]
    for p in procs:
        p.start()
    tmax, parts = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert tmax == 2.0
    w, h, spp, depth = 40, 22, 4, 20
    full = _render_rows(list(range(h)), w, h, spp, depth)
    if scaling == "strong":
        assert np.array_equal(gather_rows(h, w, parts), full)
    else:
        assert all(len(r) == h for r, _ in parts)
        both = _render_rows(list(range(h)), w, h, 2 * spp, depth)
        avg = (parts[0][1] + parts[1][1]) / 2
        assert np.allclose(avg, both, atol=2e-6)
        assert not np.array_equal(parts[0][1], parts[1][1])


def test_bench_defaults_to_row_tile_strong_scaling(monkeypatch):
    """bench.py's N-GPU default is north_star's row-tile shard (strong
    scaling): rank r of N renders tiles r, r + N, ... of the one frame."""
    import importlib
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2"])
    sys.path.insert(0, str(ROOT))
    bench = importlib.import_module("bench")
    a = bench.parse()
    assert a.scaling == "strong" and a.workload == "c1"
    assert (a.steps, a.warmup) == (100, 5)   # c1: a ~0.6 s timed GPU region
    monkeypatch.setattr(sys, "argv", ["bench.py", "--workload", "c4"])
    b = bench.parse()
    assert (b.steps, b.warmup) == (5, 1)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2"])
    from rtclj.shard import shard_params
    p0 = shard_params(2, 0, 1200, 675, 100, 50, scaling=a.scaling)
    p1 = shard_params(2, 1, 1200, 675, 100, 50, scaling=a.scaling)
    assert (p0["tile_first"], p1["tile_first"], p0["tile_step"]) == (0, 1, 2)
    assert set(bench.WORKLOADS) == {"c1", "c2", "c3", "c4"}
