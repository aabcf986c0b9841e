"""Parity at BASELINE.json's full sizes: C1-C5 scenes and frames exactly
as bench.py builds them (rtamd.configs: Collada round trip for C2-C4, the restated
SplitBVHBuilder), rendered through the C ABI on MI355X.

Two pins per config:
  * S_strict (RT_FLAG_STRICT_MATH) against the CPU oracle on the WHOLE frame: hit ids,
    closest-hit t, float RGB and packed pixels bit for bit (RGB also within 1e-4);
  * the default arithmetic S_ref against the REFERENCE kernel itself (volumeRender.cl as
    RayTracer.cpp builds it, oracle/_ref, run in a child process) on the whole frame.
    The reference kernel has RAY_TRACE_DEPTH = 3 and the shadow ray compiled in
    (volumeRender.cl:12, 1437), so this pin renders depth 3 with shadows; the depth-1
    frames of C3/C4 are then tied to it through their first bounce (hit ids and t of a
    depth-1 frame == bounce 0 of the pinned depth-3 frame).
C4 is rendered as 2-, 4- and 8-way band shards re-interleaved by rt_assemble_bands (the
multi-GPU frame path); C5 in the wavefront mode, with and without the per-bounce ray sort.
"""
import os

import numpy as np
import pytest

from conftest import ROOT  # noqa: F401  (sys.path set-up)

pytestmark = pytest.mark.gpu

STRICT = 64          # RT_FLAG_STRICT_MATH
WAVEFRONT, WF_SORT = 8, 32
RGB_TOL = 1e-4
_cache = {}


def _config(name):
    """(scene, params, cfg) of a BASELINE config, built once per test session."""
    if name not in _cache:
        import rtamd
        from rtamd import configs
        cfg = configs.CONFIGS[name]
        mesh, bvh, _ = configs.make_scene(cfg, threads=16)
        scene = rtamd.Scene.from_mesh(mesh, bvh)
        params = rtamd.params_to_array(mesh.camera_params(cfg["w"], cfg["h"]))
        _cache.clear()   # one scene at a time (C5 holds ~2 GB of host arrays)
        _cache[name] = (scene, params, cfg)
    return _cache[name]


def _compare(gpu, ref, label):
    bad = np.argwhere(gpu["hits"] != ref["hits"])
    assert bad.size == 0, f"{label}: {len(bad)} hit ids differ, first at {bad[:3].tolist()}"
    assert np.array_equal(gpu["t"].view(np.uint32), ref["t"].view(np.uint32)), f"{label}: t differs"
    assert float(np.max(np.abs(gpu["rgb"] - ref["rgb"]))) <= RGB_TOL, f"{label}: rgb beyond 1e-4"
    assert np.array_equal(gpu["rgb"].view(np.uint32), ref["rgb"].view(np.uint32)), f"{label}: rgb not bitwise"
    assert np.array_equal(gpu["out"], ref["out"]), f"{label}: packed pixels differ"


def _reference(scene, params, w, h, tmp_path):
    from oracle import ref_ocl
    if not ref_ocl.available():
        pytest.skip("oracle/_ref (the reference kernel's code objects) not in this snapshot")
    return ref_ocl.render_subprocess(scene, params, w, h, "default", str(tmp_path))


def _banded(renderer, w, h, depth, flags, nranks, band_rows=8):
    """Every rank's bands rendered into its slot of one (nranks, slot) buffer -- what the
    RCCL gather delivers to rank 0 -- then one rt_assemble_bands launch."""
    import rtamd
    import torch
    slot = (rtamd.tiling_pixels(w, h, 0, nranks, band_rows) + 3) // 4 * 4
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        slots = torch.zeros((nranks, slot), dtype=torch.int32, device="cuda")
        frame = torch.full((h * w,), -1, dtype=torch.int32, device="cuda")
        for rank in range(nranks):
            t = rtamd.rt_tiling(rank, nranks, band_rows, 0)
            renderer.render_device(w, h, depth, flags, slots[rank].data_ptr(), tiling=t, stream=side.cuda_stream)
        rtamd.assemble_bands_device(frame.data_ptr(), slots.data_ptr(), slot, w, h, nranks, band_rows,
                                    side.cuda_stream)
    torch.cuda.synchronize()
    out = frame.cpu().numpy().view(np.uint32).copy()
    del slots, frame
    return out


@pytest.mark.parametrize("name", ["c1", "c2", "c3", "c5"])
def test_strict_matches_oracle_whole_frame(renderer, name):
    """S_strict against the CPU oracle at the config's own size, depth, flags and path."""
    from oracle import oracle
    scene, params, cfg = _config(name)
    renderer.upload(scene)
    renderer.set_params(params)
    w, h, depth = cfg["w"], cfg["h"], cfg["depth"]
    gpu = renderer.render(w, h, depth=depth, flags=cfg["flags"] | STRICT, aux=True)
    ref = oracle.render(scene, params, w, h, depth=depth, flags=cfg["flags"])
    _compare(gpu, ref, name)
    assert int((gpu["hits"][:, 0, 0] >= 0).sum()) > 0.5 * w * h or name == "c2"   # the frame is mostly scene
    if name == "c5":   # the adaptive block order's second frame, and the unsorted queues
        _compare(renderer.render(w, h, depth=depth, flags=cfg["flags"] | STRICT, aux=True), ref, "c5 (2nd frame)")
        _compare(renderer.render(w, h, depth=depth, flags=WAVEFRONT | STRICT, aux=True), ref, "c5 unsorted")


@pytest.mark.parametrize("name", ["c1", "c2", "c3", "c5"])
def test_default_math_matches_reference_kernel(renderer, name, tmp_path):
    """S_ref (rt_render's default arithmetic) against the reference kernel as its host
    builds it, the whole frame at depth 3 with shadows (the reference's compiled-in
    setting), on the config's scene and camera; C5 through its wavefront path, sorted and unsorted."""
    scene, params, cfg = _config(name)
    w, h = cfg["w"], cfg["h"]
    ref = _reference(scene, params, w, h, tmp_path)
    renderer.upload(scene)
    renderer.set_params(params)
    flags = cfg["flags"] & (WAVEFRONT | WF_SORT)
    out = renderer.render(w, h, depth=3, flags=flags)
    nd = int(np.sum(out != ref))
    print(f"{name}: S_ref depth 3 vs reference kernel: {nd} of {out.size} pixels differ")
    assert nd == 0
    assert int(np.sum(renderer.render(w, h, depth=3, flags=flags ^ WAVEFRONT if flags else WAVEFRONT) != ref)) == 0
    if name == "c5":   # and the unsorted wavefront
        assert int(np.sum(renderer.render(w, h, depth=3, flags=WAVEFRONT) != ref)) == 0
    if cfg["depth"] == 1:
        # the depth-1 frame's rays are bounce 0 of the pinned depth-3 frame
        d3 = renderer.render(w, h, depth=3, aux=True)
        d1 = renderer.render(w, h, depth=1, flags=cfg["flags"], aux=True)
        assert np.array_equal(d1["hits"][:, 0, 0], d3["hits"][:, 0, 0])
        assert np.array_equal(d1["t"][:, 0].view(np.uint32), d3["t"][:, 0].view(np.uint32))
        if not cfg["flags"] & 1:   # with the shadow ray: the same shadow hits
            assert np.array_equal(d1["hits"][:, 0, 1], d3["hits"][:, 0, 1])
        # the benched pixels themselves: with the shadow ray (C3) on every pixel whose depth-3 trace
        # stopped after one hit; primary-only (C2, RT_FLAG_NO_SHADOW) where, in addition, that hit's
        # shadow any-hit missed (coefficient 1 in both frames)
        _pin_depth1_pixels(name, d3, d1["out"], ref, unshadowed=bool(cfg["flags"] & 1))


def _pin_depth1_pixels(label, d3, out1, ref, unshadowed=False):
    """The benched depth-1 pixels themselves against the reference kernel.  The reference
    always traces RAY_TRACE_DEPTH = 3 bounces (volumeRender.cl:12), but a pixel whose reflected
    ray misses ends with ray_depth = 1, and its packed colour is then color / 1 * shadow / 1
    (volumeRender.cl:1519-1546): exactly the depth-1 frame's.  So on every pixel where the
    pinned depth-3 frame stopped after its first hit (or its primary ray missed: black in
    both) the depth-1 frame must equal the reference kernel's packed pixel.
    unshadowed (a primary-only depth-1 frame, RT_FLAG_NO_SHADOW: its shadow coefficient is
    1): only where the depth-3 frame's bounce-0 shadow any-hit also missed (coefficient 1
    there too, volumeRender.cl:1437-1460)."""
    h0, h1 = d3["hits"][:, 0, 0], d3["hits"][:, 1, 0]
    one_hit = (h0 >= 0) & (h1 < 0)
    if unshadowed:
        one_hit &= d3["hits"][:, 0, 1] < 0
    subset = one_hit | (h0 < 0)
    nd = int(np.sum(out1[subset] != ref[subset]))
    print(f"{label}: S_ref depth-1 frame vs reference kernel on {int(one_hit.sum())} one-hit"
          f"{' unshadowed' if unshadowed else ''} pixels (+{int((h0 < 0).sum())} primary misses) of "
          f"{out1.size} ({int((h0 >= 0).sum())} scene pixels): {nd} differ")
    assert nd == 0
    if label.startswith(("c2", "c3", "c4")):   # most reflected rays leave the scene (C1's room keeps them)
        assert one_hit.sum() > 0.5 * (h0 >= 0).sum(), "the subset covers most of the scene's pixels"


@pytest.mark.parametrize("nranks", [2, 4, 8])
def test_c4_band_shards_assemble_to_oracle_frame(renderer, nranks):
    """C4 (the C3 scene at 4K) as N-way band shards -> rt_assemble_bands == the oracle's frame."""
    from oracle import oracle
    scene, params, cfg = _config("c4")
    w, h, depth = cfg["w"], cfg["h"], cfg["depth"]
    key = ("c4_oracle",)
    if key not in _cache:
        _cache[key] = oracle.render(scene, params, w, h, depth=depth, flags=cfg["flags"], aux=False)["out"]
    renderer.upload(scene)
    renderer.set_params(params)
    out = _banded(renderer, w, h, depth, cfg["flags"] | STRICT, nranks)
    assert np.array_equal(out, _cache[key]), f"{int(np.sum(out != _cache[key]))} pixels differ"


def test_c4_default_math_shards_match_reference_kernel(renderer, tmp_path):
    """C4 at depth 3 in the default arithmetic, rendered as 8 band shards and assembled,
    against the reference kernel's 4K frame."""
    scene, params, cfg = _config("c4")
    w, h = cfg["w"], cfg["h"]
    ref = _reference(scene, params, w, h, tmp_path)
    renderer.upload(scene)
    renderer.set_params(params)
    out = _banded(renderer, w, h, 3, 0, 8)
    assert int(np.sum(out != ref)) == 0
    # the benched depth-1 arithmetic, as the same 8 assembled shards, on the pixels whose
    # depth-3 trace stopped after one hit
    d3 = renderer.render(w, h, depth=3, aux=True)
    assert np.array_equal(d3["out"], ref)
    _pin_depth1_pixels("c4 (8 shards)", d3, _banded(renderer, w, h, 1, 0, 8), ref)
