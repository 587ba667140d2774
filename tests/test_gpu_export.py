"""Path export for split launches (KArgs xq, trace_kernel<..., SWEEP>,
DESIGN.md §3.1): with RTCLJ_EXPORT=1 a split launch's waves write their last
paths out as records once their batches are spent and leave; a sweep launch
runs the records to their ends and adds their colours to the split sums in
HBM.  Integer sums: the frame's bits may not change.  Every case here is
compared with the same launch without export (itself pinned by
test_gpu_schedule.py / test_gpu_parity.py), into NaN-filled buffers, and
rt_export_stats shows that records were written (the export ran)."""
import ctypes as C

import numpy as np
import pytest

from test_gpu_schedule import _launch, _render, env  # noqa: F401  (the module's scene fixture)

pytestmark = pytest.mark.gpu


def _exported(env, stream=None):
    from rtclj._lib import check, lib
    torch = env[2]
    s = stream or torch.cuda.current_stream()
    st = (C.c_uint64 * 2)()
    check(lib.rt_export_stats(env[1], C.c_void_p(s.cuda_stream), st))
    return int(st[0]), int(st[1])


@pytest.fixture
def knobs(monkeypatch):
    def set_knobs(**kw):
        for k, v in kw.items():
            if v is None:
                monkeypatch.delenv(k, raising=False)
            else:
                monkeypatch.setenv(k, str(v))
    yield set_knobs
    for k in ("RTCLJ_EXPORT", "RTCLJ_EXPORT_LIM", "RTCLJ_SPLIT", "RTCLJ_SPLIT_PLAN"):
        monkeypatch.delenv(k, raising=False)


@pytest.mark.parametrize("spp", [1, 2, 7, 37, 100])
@pytest.mark.parametrize("lim", [64, 16, 1])
def test_export_is_bit_exact(env, knobs, spp, lim):
    """Split launches with export (limits: every path once the batches are
    spent, 16, 1) give the unexported split launch's bits, in plain and
    recorded order; spp 1 / 2 with more splits than samples (clamped; spp 1
    runs unsplit, without export)."""
    from rtclj import scenes
    w, h = 90, 53
    cam = scenes.cover_camera(w, h)
    knobs(RTCLJ_SPLIT=1, RTCLJ_EXPORT=None)
    want = _launch(env, cam, w, h, spp)
    assert not np.isnan(want).any()
    _exported(env)
    for k in (2, 3, 5, 64):
        knobs(RTCLJ_SPLIT=k, RTCLJ_EXPORT=1, RTCLJ_EXPORT_LIM=lim)
        for _ in range(2):   # the second launch runs the recorded order
            got = _launch(env, cam, w, h, spp)
            assert np.array_equal(got, want), (spp, lim, k)
        n, rec = _exported(env)
        assert n == (2 if min(k, spp) > 1 else 0), (spp, k)   # (spp 1: no split, nothing to export)
        if lim == 64 and spp >= 7:
            assert rec > 0, (spp, k)    # the sweep had paths to run


def test_export_shards_realm_stripes_and_plans(env, knobs):
    """Interleaved row-tile shards, a sample stripe (sample_begin), realm
    semantics and cost-balanced splits (RTCLJ_SPLIT_PLAN=1) with export:
    the unexported bits."""
    from rtclj import scenes
    from rtclj._lib import RT_FLAG_REALM
    sc = env[0]
    w, h = 120, 67
    cam = scenes.cover_camera(w, h)
    knobs(RTCLJ_SPLIT=1, RTCLJ_EXPORT=None)
    full = _render(sc, cam, w, h, 12)
    stripe = _launch(env, cam, w, h, 5, sample_begin=7)
    realm = _render(sc, cam, w, h, 6, flags=RT_FLAG_REALM)
    for k in (4, 12):
        knobs(RTCLJ_SPLIT=k, RTCLJ_EXPORT=1)
        for f in range(3):
            part = _launch(env, cam, w, h, 12, row_tile=8, tile_first=f, tile_step=3)
            rows = np.concatenate([np.arange(t, min(t + 8, h)) for t in range(8 * f, h, 24)])
            assert np.array_equal(part, full[rows]), (k, f)
        assert np.array_equal(_launch(env, cam, w, h, 5, sample_begin=7), stripe), k
        assert np.array_equal(_render(sc, cam, w, h, 6, flags=RT_FLAG_REALM), realm), k
    knobs(RTCLJ_SPLIT=4, RTCLJ_EXPORT=1, RTCLJ_SPLIT_PLAN=1)
    for _ in range(3):
        assert np.array_equal(_launch(env, cam, w, h, 12), full)


def test_export_c1_shards_full_spp(env, knobs):
    """C1's 8- and 4-GPU shards at full spp (the launches export is for:
    the automatic 3-way split), twice each, and frames in flight on two
    streams (RT_FLAG_STREAMED): rt_render's rows; the segment and sample
    counters equal the unexported launch's."""
    from rtclj import scenes
    from rtclj._lib import RT_FLAG_STREAMED, check, lib, rt_params
    from rtclj.shard import shard_params, shard_rows
    sc, ds, torch = env
    w, h, spp = 1200, 675, 100
    cam = scenes.cover_camera(w, h)
    full = _render(sc, cam, w, h, spp)

    def launch(p, stream, counters=None):
        n = check(lib.rt_rows_out(C.byref(p)))
        with torch.cuda.stream(stream):
            out = torch.full((n * w * 3,), float("nan"), dtype=torch.float32, device="cuda")
        rc = lib.rt_launch(ds, C.byref(cam), C.byref(p), C.c_void_p(out.data_ptr()),
                           None if counters is None else C.c_void_p(counters.data_ptr()), C.c_void_p(stream.cuda_stream))
        assert rc == 0, lib.rt_last_error()
        return out, n

    s0 = torch.cuda.current_stream()
    _exported(env, s0)   # (reset: the earlier tests' launches on this stream)
    for world in (8, 4):
        rank = world - 1
        p = rt_params(**shard_params(world, rank, w, h, spp, 50, 1, "strong"))
        want = full[shard_rows(h, 8, rank, world)]
        cnt = {}
        for xp in (None, 1, 1):
            knobs(RTCLJ_EXPORT=xp)
            c = torch.zeros(2, dtype=torch.int64, device="cuda")
            out, n = launch(p, s0, c)
            torch.cuda.synchronize()
            assert np.array_equal(out.cpu().numpy().reshape(n, w, 3), want), (world, xp)
            cnt.setdefault(xp, []).append(tuple(c.cpu().tolist()))
        assert cnt[1][0] == cnt[1][1] == cnt[None][0], world
        ne, rec = _exported(env, s0)
        assert ne == 2 and rec > 0, (world, ne, rec)
        # frames in flight on two streams, never synchronised in between
        knobs(RTCLJ_EXPORT=1)
        p.flags |= RT_FLAG_STREAMED
        streams = [torch.cuda.Stream() for _ in range(2)]
        frames = [launch(p, streams[f % 2]) for f in range(4)]
        torch.cuda.synchronize()
        for f, (out, n) in enumerate(frames):
            assert np.array_equal(out.cpu().numpy().reshape(n, w, 3), want), (world, f)
        for s in streams:
            assert _exported(env, s)[0] == 2, world
