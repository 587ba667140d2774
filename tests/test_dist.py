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
    # value is single-frame throughput at every N: the same
    # basis at N = 1 and N > 1, the pipelined one timed beside it
    assert a.inflight == 1 and b.inflight == 1 and a.pipelined == "auto"


def _summary_worker(rank, world, port, q):
    sys.path[:0] = [str(ROOT), str(ROOT / "raytracing-clj_amd")]
    import torch.distributed as dist
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # a rank's own record as bench.main() builds it (times of a made-up frame)
    mine = {"rank": rank, "device": rank, "device_uuid": f"GPU-{rank:02d}", "pci_bus_id": 0x10 + rank,
            "elapsed_s": 1.0 + rank, "elapsed_barrier_s": 1.1 + rank, "kernel_ms_avg": 10.0, "rows": 80 + rank,
            "samples": 1000, "ms_per_frame": 10.0 * (1 + rank), "other_elapsed_s": 0.5, "other_samples": 1000}
    per_rank = [None] * world
    dist.all_gather_object(per_rank, mine)
    if rank == 0:
        q.put(bench.rank_summary(per_rank, 1, 2, 100, 5))
    dist.barrier()
    dist.destroy_process_group()


def test_bench_line_names_its_basis_and_devices():
    """The cross-rank part of bench.py's line, from records gathered over a
    world-size-2 gloo job: both bases (single_frame, pipelined) with value =
    samples of all ranks / the slowest rank's time, scaling_basis naming the
    one `value` is, and each rank's device ordinal / UUID / PCI bus."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_summary_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    s = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert s["scaling_basis"] == "single_frame"
    assert s["single_frame"]["value"] == pytest.approx(2000 / 2.0 / 1e6)   # max elapsed over ranks
    assert s["pipelined"]["value"] == pytest.approx(2000 / 0.5 / 1e6) and s["pipelined"]["streams_per_rank"] == 2
    pr = s["per_rank"]
    assert pr["device"] == [0, 1] and pr["device_uuid"] == ["GPU-00", "GPU-01"] and pr["distinct_devices"] == 2
    assert pr["rows"] == [80, 81] and pr["imbalance"] == pytest.approx(20 / 15)
