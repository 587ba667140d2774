"""write-color! on the device (rt_quantize_device, rt_render_u8).

The device quantiser turns a channel into its byte by counting the 255 float
thresholds between bytes (rt_internal.h quantize_thresholds).  Its bytes must
equal rt_quantize's (write-color!, raytracing.clj:19-26) for EVERY float:
here every threshold and the 64 floats on either side of it, the specials
(NaN payloads of both signs, infinities, signed zeros, denormals, negatives)
and a million random bit patterns; then whole frames through rt_render_u8,
one device and split into interleaved shards with a short last row tile,
against rt_quantize of rt_render's floats.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import pytest
import torch  # noqa: F401  (before rtclj: torch's HIP runtime must serve the process, conftest.gpu_lib)

gpu = pytest.mark.gpu


def _host_q(x):
    from rtclj import raytracing as R
    return R.write_color(np.ascontiguousarray(x, np.float32))


def _thresholds():
    """t[q] = the smallest positive float whose byte is >= q, by a binary
    search over bit patterns with rt_quantize itself (all 255 at once)."""
    lo = np.zeros(255, np.uint32)
    hi = np.full(255, 0x7F800000, np.uint32)
    want = np.arange(1, 256)
    while np.any(hi - lo > 1):
        mid = (lo + (hi - lo) // 2).astype(np.uint32)
        ge = _host_q(mid.view(np.float32)).astype(np.int64) >= want
        hi = np.where(ge, mid, hi)
        lo = np.where(ge, lo, mid)
    return hi


def _device_q(x):
    import torch
    from rtclj._lib import lib
    d_in = torch.from_numpy(np.ascontiguousarray(x, np.float32)).cuda()
    d_out = torch.empty(d_in.numel(), dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    rc = lib.rt_quantize_device(C.c_void_p(d_in.data_ptr()), C.c_void_p(d_out.data_ptr()), d_in.numel(),
                                C.c_void_p(s.cuda_stream))
    assert rc == 0, lib.rt_last_error()
    torch.cuda.synchronize()
    return d_out.cpu().numpy()


def test_threshold_count_is_rt_quantize():
    """(CPU) The device's rule -- a channel's byte is the number of
    thresholds <= it, an 8-step search -- restated in numpy over the
    thresholds derived from rt_quantize, equals rt_quantize on random bit
    patterns and the specials."""
    thr = np.concatenate([[np.float32(-np.inf)], _thresholds().view(np.float32)])
    bits = np.random.default_rng(3).integers(0, 1 << 32, size=1 << 18, dtype=np.uint64).astype(np.uint32)
    bits = np.concatenate([bits, np.array([0x7FC00000, 0xFFC00000, 0x7F800000, 0xFF800000, 0, 0x80000000, 1],
                                          np.uint32)])
    x = bits.view(np.float32)
    b = np.zeros(x.size, np.int64)
    with np.errstate(invalid="ignore"):
        for step in (128, 64, 32, 16, 8, 4, 2, 1):
            b = np.where(thr[b + step] <= x, b + step, b)
    assert np.array_equal(b.astype(np.uint8), _host_q(x))


@gpu
def test_quantize_device_every_boundary_and_special(gpu_lib):
    thr = _thresholds()
    near = (thr[:, None].astype(np.int64) + np.arange(-64, 65)[None, :]).reshape(-1)
    near = near[(near >= 0) & (near <= 0x7F800000)].astype(np.uint32)
    specials = np.array([0x7FC00000, 0xFFC00000, 0x7F800001, 0x7FFFFFFF, 0xFFFFFFFF, 0x7F800000, 0xFF800000,
                         0x00000000, 0x80000000, 0x00000001, 0x007FFFFF, 0x80000001, 0x3F800000, 0xBF800000,
                         0x3F7FBE77, 0x3F7FFFFF, 0x7F7FFFFF, 0xFF7FFFFF], np.uint32)
    rnd = np.random.default_rng(7).integers(0, 1 << 32, size=1 << 20, dtype=np.uint64).astype(np.uint32)
    bits = np.concatenate([near, specials, rnd])
    x = bits.view(np.float32)
    host = _host_q(x)
    dev = _device_q(x)
    bad = np.nonzero(host != dev)[0]
    assert bad.size == 0, [(hex(int(bits[i])), int(host[i]), int(dev[i])) for i in bad[:8]]
    # every byte value occurs, and each threshold is where its byte starts
    assert set(np.unique(host[:near.size]).tolist()) == set(range(256))
    assert np.array_equal(_host_q(thr.view(np.float32)), np.arange(1, 256, dtype=np.uint8))


@gpu
@pytest.mark.parametrize("n", [0, 1, 3, 255, 257, 4096 * 256 + 5])
def test_quantize_device_lengths(gpu_lib, n):
    """Ragged lengths, the empty one and more channels than the grid covers
    in one pass (grid-stride loop)."""
    x = np.random.default_rng(n).uniform(-0.1, 1.2, size=n).astype(np.float32)
    assert np.array_equal(_device_q(x), _host_q(x))


@gpu
def test_quantize_device_arguments(gpu_lib):
    from rtclj._lib import lib
    assert lib.rt_quantize_device(None, None, 4, None) == -1
    assert lib.rt_quantize_device(None, None, 0, None) == 0


@gpu
@pytest.mark.parametrize("ndev,height", [(1, 225), (3, 69), (8, 61)])
def test_render_u8_equals_quantized_render(gpu_lib, ndev, height):
    """rt_render_u8 == rt_quantize(rt_render) on the cover scene, one shard
    and interleaved shards on device 0 (the strided byte copies, a short
    last row tile)."""
    from rtclj import raytracing as R, scenes
    from rtclj._lib import RT_FLAG_SHARDS_ON_DEVICE0
    w = 400 if height == 225 else 104
    sc = scenes.cover(11)
    cam = scenes.cover_camera(w, height)
    kw = dict(spp=4, seed=5, n_devices=ndev, flags=RT_FLAG_SHARDS_ON_DEVICE0 if ndev > 1 else 0)
    lin = R.render(sc, cam, w, height, **kw)
    st = {}
    q = R.render(sc, cam, w, height, u8=True, stats=st, **kw)
    assert q.dtype == np.uint8 and q.shape == (height, w, 3)
    assert np.array_equal(q, R.write_color(lin))
    assert st["n_devices"] == ndev
    # the reference scene at the -main resolution, a row range
    ref = R.Scene.from_bodies(R.hittables)
    cam2 = R.camera(400, 225, **R.REFERENCE_CAMERA)
    a = R.render(ref, cam2, 400, 225, spp=2, rows=(37, 190), u8=True)
    assert np.array_equal(a, R.write_color(R.render(ref, cam2, 400, 225, spp=2, rows=(37, 190))))
