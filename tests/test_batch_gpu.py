"""rt_render_device_batch: several depth-1 frames in ONE launch (throughput mode, DESIGN.md 7;
the reference renders one frame per raytrace_gpgpu, RayTracer.cpp:330-344).

Bar: every frame of a batch equals rt_render_device's frame for its own camera, bit for bit --
in the three math modes, with and without the shadow ray, for 1..RT_MAX_BATCH frames of
different cameras, on the first call of a geometry (the static order, a tile of every frame side
by side) and on later calls (the longest-first order built over all frames' blocks), for a band
of a multi-GPU tiling, and with a frame stride above the frame size (the gap untouched); C2 and
C3 at full size; and depth 2-3 in the wavefront mode (one bounce-0 launch for all frames, then one
launch per bounce over all frames' queues), contiguous or a stride apart, C5 at full size.  Argument errors are refused before
anything is enqueued."""
import numpy as np
import pytest

from conftest import load_golden

pytestmark = pytest.mark.gpu

STRICT, HW, NO_SHADOW, WAVEFRONT, WF_SORT, STATIC_ORDER, EXACT_DIV = 64, 2, 1, 8, 32, 16, 4


def _cams(mesh, w, h, k):
    return [mesh.camera_params(w, h, extra_alpha=0.07 * i, extra_beta=0.03 * i) for i in range(k)]


def _singles(renderer, w, h, flags, cams, tiling=None, npx=None, depth=1):
    import torch
    npx = npx or w * h
    out = []
    for p in cams:
        renderer.set_params(p)
        dev = torch.full((npx,), -1, dtype=torch.int32, device="cuda")
        renderer.render_device(w, h, depth, flags, dev.data_ptr(), tiling=tiling)
        torch.cuda.synchronize()
        out.append(dev.cpu().numpy().view(np.uint32).copy())
    return out


def _batch(renderer, w, h, flags, cams, stride, npx, tiling=None, depth=1):
    import torch
    out = torch.full((len(cams) * stride,), -7, dtype=torch.int32, device="cuda")
    renderer.render_device_batch(w, h, depth, flags, cams, out.data_ptr(), stride, tiling=tiling)
    torch.cuda.synchronize()
    o = out.cpu().numpy().view(np.uint32)
    frames = [o[i * stride:i * stride + npx].copy() for i in range(len(cams))]
    gaps = [o[i * stride + npx:(i + 1) * stride] for i in range(len(cams))]
    return frames, all(bool(np.all(g.view(np.int32) == -7)) for g in gaps)


@pytest.mark.parametrize("k", [1, 2, 3, 8])
def test_batch_frames_equal_single_renders(renderer, k):
    import rtamd
    d = load_golden("knot16k")
    renderer.upload(rtamd.Scene.from_arrays(d))
    mesh = rtamd.Mesh.torus_knot(128, 64)
    for w, h in ((int(d["w"]), int(d["h"])), (123, 77), (640, 360)):
        cams = _cams(mesh, w, h, k)
        for flags in (0, NO_SHADOW, STRICT, STRICT | NO_SHADOW, HW, STATIC_ORDER, EXACT_DIV):
            want = _singles(renderer, w, h, flags, cams)
            for call in range(3):   # call 0: static order; then the adaptive order of all frames
                got, gaps_ok = _batch(renderer, w, h, flags, cams, w * h + 37, w * h)
                assert gaps_ok, (k, w, h, flags, call)
                for i in range(k):
                    assert np.array_equal(got[i], want[i]), (k, w, h, flags, call, i, int(np.sum(got[i] != want[i])))
    t, _ = renderer.last_timing()
    assert t > 0.0


@pytest.mark.parametrize("k", [1, 2, 3, 8])
def test_wavefront_batch_frames_equal_single_renders(renderer, k):
    """Depth 3 in the wavefront mode: bounce 0 of every frame in one launch, then each bounce
    launch over all frames' queues (sorted and unsorted), every ray finishing in its own frame."""
    import rtamd
    d = load_golden("knot16k")
    renderer.upload(rtamd.Scene.from_arrays(d))
    mesh = rtamd.Mesh.torus_knot(128, 64)
    for w, h in ((int(d["w"]), int(d["h"])), (123, 77), (640, 360)):
        cams = _cams(mesh, w, h, k)
        for flags in (WAVEFRONT, WAVEFRONT | WF_SORT, WAVEFRONT | STRICT, WAVEFRONT | WF_SORT | NO_SHADOW, WAVEFRONT | HW,
                      WAVEFRONT | WF_SORT | STATIC_ORDER):
            want = _singles(renderer, w, h, flags, cams, depth=3)
            for call in range(3):   # contiguous frames, then frames a stride apart (the gaps untouched)
                stride = w * h + (0 if call < 2 else 37)
                got, gaps_ok = _batch(renderer, w, h, flags, cams, stride, w * h, depth=3)
                assert gaps_ok
                for i in range(k):
                    assert np.array_equal(got[i], want[i]), (k, w, h, flags, call, i, int(np.sum(got[i] != want[i])))
    # depth 2, and a band of a 2-way tiling
    w, h = 333, 201
    t = rtamd.rt_tiling(1, 2, 8, 0)
    npx = rtamd.tiling_pixels(w, h, 1, 2, 8)
    cams = _cams(mesh, w, h, 3)
    want = _singles(renderer, w, h, WAVEFRONT | WF_SORT, cams, tiling=t, npx=npx, depth=2)
    got, _ = _batch(renderer, w, h, WAVEFRONT | WF_SORT, cams, npx, npx, tiling=t, depth=2)
    for i in range(3):
        assert np.array_equal(got[i], want[i]), i
    # the band of a 3-way tiling in buffers padded to the largest rank's (bench.py at N > 1: a
    # rank with fewer bands keeps the others' slot size)
    t = rtamd.rt_tiling(2, 3, 8, 0)
    npx = rtamd.tiling_pixels(w, h, 2, 3, 8)
    cap = (rtamd.tiling_pixels(w, h, 0, 3, 8) + 3) // 4 * 4
    assert cap > npx
    want = _singles(renderer, w, h, WAVEFRONT | WF_SORT, cams, tiling=t, npx=npx, depth=3)
    got, gaps_ok = _batch(renderer, w, h, WAVEFRONT | WF_SORT, cams, cap, npx, tiling=t, depth=3)
    assert gaps_ok
    for i in range(3):
        assert np.array_equal(got[i], want[i]), i


def test_batch_band_tiling_and_mixed_calls(renderer):
    """A rank's bands (rt_tiling) in a batch; batches of other sizes and single frames on the
    same stream in between (each keeps its own block order)."""
    import rtamd
    d = load_golden("knot16k")
    renderer.upload(rtamd.Scene.from_arrays(d))
    mesh = rtamd.Mesh.torus_knot(128, 64)
    w, h = 333, 201
    t = rtamd.rt_tiling(1, 3, 8, 0)
    npx = rtamd.tiling_pixels(w, h, 1, 3, 8)
    cams = _cams(mesh, w, h, 5)
    want = _singles(renderer, w, h, 0, cams, tiling=t, npx=npx)
    for k in (5, 2, 5, 1, 4):
        got, gaps_ok = _batch(renderer, w, h, 0, cams[:k], npx, npx, tiling=t)
        assert gaps_ok
        for i in range(k):
            assert np.array_equal(got[i], want[i]), (k, i)
        # a single frame between batches
        one = _singles(renderer, w, h, 0, cams[k - 1:k], tiling=t, npx=npx)[0]
        assert np.array_equal(one, want[k - 1])


def test_batch_argument_errors(renderer):
    import rtamd
    import torch
    d = load_golden("knot16k")
    renderer.upload(rtamd.Scene.from_arrays(d))
    mesh = rtamd.Mesh.torus_knot(128, 64)
    w, h = 64, 64
    out = torch.zeros(9 * w * h, dtype=torch.int32, device="cuda")
    cams = _cams(mesh, w, h, 9)
    for args, what in (((w, h, 1, 0, cams, out.data_ptr(), w * h), "nframes"),        # 9 > RT_MAX_BATCH
                       ((w, h, 1, 0, [], out.data_ptr(), w * h), "nframes"),          # 0 frames
                       ((w, h, 3, 0, cams[:2], out.data_ptr(), w * h), "depth 1"),    # depth 3, not wavefront
                       ((w, h, 1, 0, cams[:2], out.data_ptr(), w * h - 1), "stride"),
                       ((w, h, 1, STRICT | HW, cams[:2], out.data_ptr(), w * h), "exclude")):
        with pytest.raises(rtamd.RtError) as e:
            renderer.render_device_batch(*args)
        assert e.value.code == -1 and what in str(e.value), (what, str(e.value))
    far = mesh.camera_params(w, h)
    far.scene_aabb_max.x += 1.0
    with pytest.raises(rtamd.RtError) as e:
        renderer.render_device_batch(w, h, 1, 0, [cams[0], far], out.data_ptr(), w * h)
    assert "scene boxes" in str(e.value)
    lit = mesh.camera_params(w, h)
    lit.light_pos.y += 1.0
    renderer.render_device_batch(w, h, 1, 0, [cams[0], lit], out.data_ptr(), w * h)   # depth 1: each frame's light
    with pytest.raises(rtamd.RtError) as e:
        renderer.render_device_batch(w, h, 3, WAVEFRONT, [cams[0], lit], out.data_ptr(), w * h)
    assert "one light" in str(e.value)


@pytest.mark.parametrize("name", ["c2", "c3", "c5"])
def test_batch_full_size_frames_equal_single_renders(renderer, name):
    """BASELINE C2 / C3 scenes and frames, four cameras per launch (the config's camera and
    three translated copies: eye and image plane moved together), against one
    rt_render_device frame per camera."""
    import rtamd
    from test_fullsize_gpu import _config
    scene, params, cfg = _config(name)
    renderer.upload(scene)
    w, h, flags, depth = cfg["w"], cfg["h"], cfg["flags"], cfg["depth"]
    cams = []
    for i in range(4):
        p = np.array(params, np.float32).copy()
        dv = np.float32(0.75 * i) * np.array([1.0, 0.5, -0.25], np.float32)
        p[8:11] += dv     # c: the image plane's origin
        p[12:15] += dv    # campos
        cams.append(rtamd.array_to_params(p))
    want = _singles(renderer, w, h, flags, cams, depth=depth)
    assert not np.array_equal(want[0], want[1])
    for call in range(2):
        got, gaps_ok = _batch(renderer, w, h, flags, cams, w * h, w * h, depth=depth)
        assert gaps_ok
        for i in range(4):
            assert np.array_equal(got[i], want[i]), (name, call, i, int(np.sum(got[i] != want[i])))
