"""Unit checks of the oracle's restated helpers against hand-derived values and
an independent numpy restatement (test infrastructure checks itself)."""
import ctypes as C

import numpy as np

from oracle import oracle


def _f(a):
    a = np.ascontiguousarray(a, np.float32)
    return a, a.ctypes.data_as(C.c_void_p)


def test_rgb_to_int_bgr_pack_clamp_truncate():
    L = oracle.lib()
    # volumeRender.cl:186-195: clamp to [0,255], truncate, b<<16 | g<<8 | r
    assert L.oracle_rgb_to_int(255.0, 0.0, 0.0) == 0x0000FF
    assert L.oracle_rgb_to_int(0.0, 0.0, 255.0) == 0xFF0000
    assert L.oracle_rgb_to_int(12.99, 300.0, -5.0) == (0 << 16) | (255 << 8) | 12
    assert L.oracle_rgb_to_int(float("nan"), 1.5, 2.5) == (2 << 16) | (1 << 8) | 0


def test_normalize_matches_devicelib_formula():
    L = oracle.lib()
    rng = np.random.default_rng(1)
    for _ in range(200):
        v = rng.normal(size=3).astype(np.float32) * np.float32(10.0 ** rng.integers(-3, 4))
        a, pa = _f(v)
        o, po = _f(np.zeros(3))
        L.oracle_normalize(pa, po)
        # independent restatement: fma dot, then p * (float)(1/sqrt((double)l2))
        x, y, z = (np.float64(t) for t in v)
        # fma(z,z, fma(y,y, x*x)): float32 products are exact in float64, so each fma
        # is one float64 add then one rounding to float32 (double rounding ~2^-29 rare)
        xx = np.float32(x * x)
        s1 = np.float32(y * y + np.float64(xx))
        s2 = np.float32(z * z + np.float64(s1))
        inv = np.float32(1.0 / np.sqrt(np.float64(s2)))
        exp = (v * inv).astype(np.float32)
        assert np.array_equal(o.view(np.uint32), exp.view(np.uint32)), (v, o, exp)
    a, pa = _f([0.0, 0.0, 0.0])
    o, po = _f([1, 1, 1])
    L.oracle_normalize(pa, po)
    assert np.all(o == 0)


def test_ray_triangle_known_answers():
    L = oracle.lib()
    ori, po = _f([0.25, 0.25, -1.0])
    d, pd = _f([0.0, 0.0, 1.0])
    v0, p0 = _f([0.0, 0.0, 0.0])
    e1, p1 = _f([1.0, 0.0, 0.0])
    e2, p2 = _f([0.0, 1.0, 0.0])
    assert L.oracle_ray_tri(po, pd, p0, p1, p2) == 1.0
    ori2, po2 = _f([0.9, 0.9, -1.0])       # u + v > 1 -> miss
    assert L.oracle_ray_tri(po2, pd, p0, p1, p2) == -1.0
    ori3, po3 = _f([-0.1, 0.5, -1.0])      # u < 0 -> miss
    assert L.oracle_ray_tri(po3, pd, p0, p1, p2) == -1.0
    dp, pdp = _f([1.0, 0.0, 0.0])          # parallel: det = 0 -> 1/0 = inf, u = nan -> not < 0, not > 1
    r = L.oracle_ray_tri(po, pdp, p0, p1, p2)
    assert np.isnan(r) or r == -1.0


def test_counters_bytes_per_ray():
    st = {"primary": {"rays": 2, "inner": 10, "leaf": 2, "tris": 4}}
    assert oracle.bytes_per_ray(st, "primary") == (80 * 10 + 16 * 2 + 64 * 4) / 2
