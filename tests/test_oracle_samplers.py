"""The kernel's loop-free samplers (include/rt.h RT_FLAG_REJECTION_SAMPLERS;
trace_kernel.h sphere_direct / disk_direct / turn24), through their fp32
restatement in the oracle, against the reference's rejection samplers
(vec3a.clj:74-79 random-unit-vec3, :81-86 random-in-unit-disk).

The contract is the same distributions: uniform on the
unit sphere, uniform in the unit disk.  The reference draws from the
unseeded java.util.Random, so no bitwise equality with it exists; these tests
pin the distributions directly and then the renders they make:

  * turn24's (cos, sin) of 2 pi u / 2^24 against double-precision math for
    every quarter-turn boundary and a dense sweep: |error| <= 2e-7;
  * 2^20 draws of each sampler: unit length (sphere) / inside the disk;
    z, r^2 and phi uniform (chi-square over 64 bins, p > 1e-4); the second
    moments 1/3 (sphere) and 1/4 (disk) within 5 sigma; the direct and the
    rejection samplers' z and r^2 indistinguishable (two-sample
    Kolmogorov-Smirnov, p > 1e-4);
  * the reference scene rendered by the fp32 mirror with the direct samplers
    against MODE_REF64 (the Clojure path in double, rejection samplers) at
    400 spp, 200x112: 16x9 block means of the linear image within 1e-3 mean
    and 8e-3 max of each other and segments/sample within 1e-3 -- about
    twice the seed-to-seed noise floor of REF64 itself, measured 6.2e-4 /
    4.5e-3 / 1.1e-4 (the direct mirror: 6.1e-4 / 4.9e-3 / 2.3e-4); the book's
    normalised-metal control (MODE_BOOK64) is far outside (1.0e-2 / 0.18 /
    1.6e-2).
tests/test_oracle_pinning.py holds the direct mirror to the reference's own
scene.ppm with SURVEY.md §8c's tolerances as well.
"""
import os

import numpy as np
import pytest
from scipy import stats

import oracle

N = 1 << 20


def test_turn24_quarter_turns_and_sweep():
    u = np.array([0, 1 << 22, 1 << 23, 3 << 22, (1 << 21) - 1, 1 << 21, (1 << 24) - 1, 0x2aaaab, 0x555555], np.uint32)
    sweep = np.arange(0, 1 << 24, 4099, dtype=np.uint32)
    for uu in (u, sweep):
        got = oracle.turn24(uu).astype(np.float64)
        phi = 2 * np.pi * uu.astype(np.float64) / (1 << 24)
        err = np.abs(got - np.stack([np.cos(phi), np.sin(phi)], 1))
        assert err.max() <= 2e-7, (err.max(), uu[np.argmax(err.max(1))])
    # exact at the quarter turns (the signs ride on r: x = -0 at a quarter turn)
    q = oracle.turn24(np.array([0, 1 << 22, 1 << 23, 3 << 22], np.uint32), r=0.5)
    assert np.array_equal(q, np.array([[0.5, 0], [0, 0.5], [-0.5, 0], [0, -0.5]], np.float32))


def _chi2_uniform(x, lo, hi, bins=64):
    h, _ = np.histogram(x, bins=bins, range=(lo, hi))
    return stats.chisquare(h).pvalue


@pytest.fixture(scope="module")
def draws():
    return {k: oracle.sampler_draws(k, 12345, N).astype(np.float64) for k in oracle.oracle.SAMPLERS}


def test_sphere_direct_is_uniform_on_the_sphere(draws):
    d = draws["sphere_direct"]
    assert np.abs(np.linalg.norm(d, axis=1) - 1).max() <= 1e-6
    assert _chi2_uniform(d[:, 2], -1, 1) > 1e-4                           # Archimedes: z uniform
    assert _chi2_uniform(np.arctan2(d[:, 1], d[:, 0]), -np.pi, np.pi) > 1e-4
    assert _chi2_uniform(d[:, 0], -1, 1) > 1e-4                           # any axis: x uniform too
    sig = np.sqrt(4 / 45 / N)   # std of the mean of x^2 (Var x^2 = 1/5 - 1/9)
    assert (np.abs((d ** 2).mean(0) - 1 / 3) <= 5 * sig).all(), (d ** 2).mean(0)
    assert (np.abs(d.mean(0)) <= 5 * np.sqrt(1 / 3 / N)).all(), d.mean(0)


def test_disk_direct_is_uniform_in_the_disk(draws):
    d = draws["disk_direct"]
    r2 = d[:, 0] ** 2 + d[:, 1] ** 2
    assert (r2 < 1).all() and (d[:, 2] == 0).all()
    assert _chi2_uniform(r2, 0, 1) > 1e-4                                 # r^2 uniform <=> area-uniform
    assert _chi2_uniform(np.arctan2(d[:, 1], d[:, 0]), -np.pi, np.pi) > 1e-4
    sig = np.sqrt((1 / 8 - 1 / 16) / N)   # x^2 of a uniform disk point: mean 1/4, E x^4 = 1/8
    assert (np.abs((d[:, :2] ** 2).mean(0) - 1 / 4) <= 5 * sig).all()


def test_direct_and_rejection_draw_the_same_distributions(draws):
    a, b = draws["sphere_direct"], draws["sphere_rejection"]
    assert np.abs(np.linalg.norm(b, axis=1) - 1).max() <= 1e-6
    for k in range(3):
        assert stats.ks_2samp(a[:, k], b[:, k]).pvalue > 1e-4, k
    c, d = draws["disk_direct"], draws["disk_rejection"]
    assert stats.ks_2samp((c[:, :2] ** 2).sum(1), (d[:, :2] ** 2).sum(1)).pvalue > 1e-4
    assert stats.ks_2samp(c[:, 0], d[:, 0]).pvalue > 1e-4


def _blocks(img, by=9, bx=16):
    h, w = img.shape[:2]
    return np.array([[img[y * h // by:(y + 1) * h // by, x * w // bx:(x + 1) * w // bx].reshape(-1, 3).mean(0)
                      for x in range(bx)] for y in range(by)])


def _render(mode, seed, w=200, h=112, spp=400):
    from rtclj import raytracing as R
    sph, kind, mat = R.flatten64(R.hittables)
    cam = oracle.camera(w, h, **R.REFERENCE_CAMERA)
    out, _, segs, smp = oracle.render(mode, sph, kind, mat, cam, 1, w, h, spp, 50, seed=seed,
                                      nthreads=min(8, os.cpu_count() or 1))
    return _blocks(out.astype(np.float64)), segs / smp


def test_direct_mirror_renders_like_ref64():
    ref, s_ref = _render(oracle.MODE_REF64, 21)
    for mode in (oracle.MODE_MIRROR32 | oracle.DIRECT, oracle.MODE_MIRROR32 | oracle.DIRECT_SPHERE):
        got, s = _render(mode, 22)
        d = np.abs(got - ref)
        assert d.mean() <= 1e-3 and d.max() <= 8e-3 and abs(s - s_ref) / s_ref <= 1e-3, (mode, d.mean(), d.max(), s)
    book, _ = _render(oracle.MODE_BOOK64, 22)
    assert np.abs(book - ref).mean() > 5e-3


def test_direct_flag_needs_an_fp32_mode():
    from rtclj import raytracing as R
    sph, kind, mat = R.flatten64(R.hittables)
    cam = oracle.camera(8, 8, **R.REFERENCE_CAMERA)
    for bad in (oracle.MODE_REF64 | oracle.DIRECT, oracle.MODE_BOOK64 | oracle.DIRECT_DISK, oracle.MODE_MIRROR32 | 0x40):
        with pytest.raises(ValueError):
            oracle.render(bad, sph, kind, mat, cam, 1, 8, 8, 1, 5)
    a = oracle.render(oracle.MODE_REALM32 | oracle.DIRECT, sph, kind, mat, cam, 1, 8, 8, 2, 5)[0]
    assert np.isfinite(a).all()
