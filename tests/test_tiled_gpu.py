"""rt_render_tiled: one frame over n contexts of ONE process (SURVEY.md 7.5 and 8b's
multi-GPU boundary; the reference renders on one device, RayTracer.cpp:330-344, 2097-2131).

The box has one GPU, so the n contexts all sit on device 0 (the API lets a device repeat):
every context renders its 8-row bands on its own stream and writes them straight into the
host frame, as n GPUs would.  Bar: the frame equals rt_render's (same flags, every pixel), into
pageable and pinned memory, at depth 1 (the depth-1 kernel's frame-row stores) and deeper (the
band buffer + row-copy path); at full size on C3 and C4; and the default-arithmetic depth-3 C3
frame equals the reference kernel's.  rt_scene_copy gives a context another one's scene."""
import numpy as np
import pytest

from conftest import load_golden

pytestmark = pytest.mark.gpu

STRICT, WAVEFRONT, WF_SORT = 64, 8, 32


def _renderers(n):
    import rtamd
    return [rtamd.Renderer(0) for _ in range(n)]


def _close(rs):
    for r in rs:
        r.close()


@pytest.mark.parametrize("n", [2, 3, 4, 8])
def test_tiled_fixture_frames_equal_rt_render(renderer, n):
    import rtamd
    import torch
    d = load_golden("knot16k")
    scene = rtamd.Scene.from_arrays(d)
    renderer.upload(scene)
    rs = _renderers(n)
    try:
        rs[0].upload(scene)
        for r in rs[1:]:
            r.copy_scene_from(rs[0])
        for w, h in ((int(d["w"]), int(d["h"])), (123, 77), (640, 360)):
            p = rtamd.params_to_array(rtamd.Mesh.torus_knot(128, 64).camera_params(w, h))
            renderer.set_params(p)
            rs[0].set_params(p)
            for depth, flags in ((1, 0), (1, STRICT), (1, 1), (3, 0), (3, STRICT), (3, WAVEFRONT | WF_SORT), (0, 0)):
                want = renderer.render(w, h, depth=depth, flags=flags)
                got = rtamd.render_tiled(rs, w, h, depth, flags)
                assert np.array_equal(got, want), (n, w, h, depth, flags, int(np.sum(got != want)))
                pinned = torch.full((w * h,), -1, dtype=torch.int32, pin_memory=True)
                rtamd.render_tiled(rs, w, h, depth, flags, out=pinned.data_ptr())
                assert np.array_equal(pinned.numpy().view(np.uint32), want), ("pinned", n, w, h, depth, flags)
        t, _ = rs[0].last_timing()
        assert t > 0.0
    finally:
        _close(rs)


@pytest.mark.parametrize("workers", ["1", "0"])
def test_tiled_workers_and_caller_thread_agree(renderer, monkeypatch, workers):
    """ctxs[1..] on their own host threads (the default) or all enqueued by the caller in turn
    (RTAMD_TILED_WORKERS=0): the same frame as rt_render, frame after frame with the camera
    moving, the workers' threads reused across calls; every context's launch is stamped
    (rt_last_enqueue_time) within this call."""
    import time
    import rtamd
    monkeypatch.setenv("RTAMD_TILED_WORKERS", workers)
    d = load_golden("knot16k")
    scene = rtamd.Scene.from_arrays(d)
    renderer.upload(scene)
    rs = _renderers(4)
    try:
        rs[0].upload(scene)
        for r in rs[1:]:
            r.copy_scene_from(rs[0])
        w, h = 160, 96
        cam = rtamd.Camera()
        mesh = rtamd.Mesh.torus_knot(128, 64)
        for i in range(12):
            cam.add_rotate(0.05, 0.0)
            p = cam.params(mesh, w, h)
            renderer.set_params(p)
            rs[0].set_params(p)
            depth = 1 if i % 3 else 3
            want = renderer.render(w, h, depth=depth, flags=0)
            t0 = time.monotonic_ns()
            got = rtamd.render_tiled(rs, w, h, depth, 0)
            t1 = time.monotonic_ns()
            assert np.array_equal(got, want), (workers, i, int(np.sum(got != want)))
            stamps = [r.last_enqueue_time() for r in rs]
            assert all(t0 <= b <= e <= t1 for b, e in stamps), (stamps, t0, t1)
    finally:
        _close(rs)


def test_tiled_argument_and_scene_errors(renderer):
    import rtamd
    d = load_golden("knot16k")
    rs = _renderers(2)
    try:
        rs[0].upload(rtamd.Scene.from_arrays(d))
        rs[0].set_params(d["params"])
        with pytest.raises(rtamd.RtError) as e:   # ctxs[1] has no scene yet
            rtamd.render_tiled(rs, 64, 64, 1, 0)
        assert e.value.code == -3 and "ctxs[1]" in str(e.value)
        rs[1].copy_scene_from(rs[0])
        out = rtamd.render_tiled(rs, 64, 64, 1, 0)
        renderer.upload(rtamd.Scene.from_arrays(d))
        renderer.set_params(d["params"])
        assert np.array_equal(out, renderer.render(64, 64, depth=1))
        with pytest.raises(rtamd.RtError):         # the same context twice
            rtamd.render_tiled([rs[0], rs[0]], 64, 64, 1, 0)
        with pytest.raises(rtamd.RtError):         # exclusive math flags
            rtamd.render_tiled(rs, 64, 64, 1, STRICT | 2)
    finally:
        _close(rs)


def test_scene_copy_is_independent_of_its_source(renderer):
    """A copied scene stays when the source context uploads another one."""
    import rtamd
    a, b = load_golden("knot16k"), load_golden("hf40k")
    rs = _renderers(2)
    try:
        rs[0].upload(rtamd.Scene.from_arrays(a))
        rs[1].copy_scene_from(rs[0])
        rs[0].upload(rtamd.Scene.from_arrays(b))
        w, h = int(a["w"]), int(a["h"])
        rs[1].set_params(a["params"])
        renderer.upload(rtamd.Scene.from_arrays(a))
        renderer.set_params(a["params"])
        assert np.array_equal(rs[1].render(w, h, depth=3, flags=STRICT), renderer.render(w, h, depth=3, flags=STRICT))
    finally:
        _close(rs)


def _config(name):
    from test_fullsize_gpu import _config as cfg
    return cfg(name)


@pytest.mark.parametrize("name,ns", [("c3", (2, 4, 8)), ("c4", (2, 8))])
def test_tiled_full_size_equals_rt_render(renderer, name, ns):
    """C3 (1080p) and C4 (4K) depth-1 frames (the benched configs) over 2/4/8 contexts."""
    import rtamd
    scene, params, cfg = _config(name)
    w, h, depth, flags = cfg["w"], cfg["h"], cfg["depth"], cfg["flags"]
    renderer.upload(scene)
    renderer.set_params(params)
    want = renderer.render(w, h, depth=depth, flags=flags)
    rs = _renderers(max(ns))
    try:
        rs[0].upload(scene)
        rs[0].set_params(params)
        for r in rs[1:]:
            r.copy_scene_from(rs[0])
        for n in ns:
            got = rtamd.render_tiled(rs[:n], w, h, depth, flags)
            assert np.array_equal(got, want), (name, n, int(np.sum(got != want)))
    finally:
        _close(rs)


def test_tiled_c3_depth3_matches_reference_kernel(renderer, tmp_path):
    """The reference's compiled-in setting (depth 3 with shadows, default arithmetic) on C3,
    over 4 contexts, against the reference kernel itself."""
    import rtamd
    from test_fullsize_gpu import _reference
    scene, params, cfg = _config("c3")
    w, h = cfg["w"], cfg["h"]
    ref = _reference(scene, params, w, h, tmp_path)
    rs = _renderers(4)
    try:
        rs[0].upload(scene)
        rs[0].set_params(params)
        for r in rs[1:]:
            r.copy_scene_from(rs[0])
        for flags in (0, WAVEFRONT | WF_SORT):
            got = rtamd.render_tiled(rs, w, h, 3, flags)
            assert int(np.sum(got != ref)) == 0, flags
    finally:
        _close(rs)


def test_grouped_render_is_one_timing_entry(renderer):
    """rt_render into pageable memory renders row groups on several streams; its timing entry
    spans the whole frame (rt_last_timing / rt_timing_average), not one group."""
    import torch
    import rtamd
    d = load_golden("knot16k")
    renderer.upload(rtamd.Scene.from_arrays(d))
    w, h = 1024, 720
    renderer.set_params(d["params"])
    dev = torch.zeros(w * h, dtype=torch.int32, device="cuda")
    for _ in range(3):
        renderer.render_device(w, h, 1, 0, dev.data_ptr())
    torch.cuda.synchronize()
    whole, _ = renderer.timing_average(3)
    for _ in range(3):
        renderer.render(w, h, depth=1)
    t_last, _ = renderer.last_timing()
    t_avg, _ = renderer.timing_average(3)
    # four row groups of a whole-frame render run concurrently: the frame's span is close to one
    # whole-frame launch, while one group alone does a quarter of its work
    assert t_last >= 0.6 * whole and t_avg >= 0.6 * whole, (t_last, t_avg, whole)
