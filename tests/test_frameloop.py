"""Headless frame loop: lib/rt_frameloop drives the C ABI as the
reference's GLUT loop does (updateCamera + render per frame, RayTracer.cpp:284-293;
orbit drag via Camera::add_rotate, :553-565) and dumps PPM frames."""
import json
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOL = os.path.join(ROOT, "real-time-opencl-raytracer_amd", "lib", "rt_frameloop")


def _read_ppm(path):
    with open(path, "rb") as f:
        data = f.read()
    parts = data.split(b"\n", 3)
    w, h = map(int, parts[1].split())
    return np.frombuffer(parts[3], np.uint8).reshape(h, w, 3)


def test_tool_is_built_and_checks_arguments():
    assert os.access(TOOL, os.X_OK), "build() must produce lib/rt_frameloop"
    for bad in (["--width", "0"], ["--gpus", "0"], ["--gpus", "65"], ["--devices", "0,x"], ["--devices", ""]):
        r = subprocess.run([TOOL, *bad], capture_output=True, text=True, timeout=60)
        assert r.returncode == 2 and "usage" in r.stderr, bad


def test_camera_orbit_matches_repeated_add_rotate():
    """rtamd.Camera accumulates add_rotate calls in float exactly as Camera.cpp:26-46."""
    import rtamd
    m = rtamd.Mesh.cornell()
    c = rtamd.Camera()
    for _ in range(3):
        c.add_rotate(0.01, 0.0)
    single = rtamd.params_to_array(m.camera_params(64, 48, extra_alpha=0.01))
    assert not np.array_equal(rtamd.params_to_array(c.params(m, 64, 48)), single)  # three calls != one call
    c2 = rtamd.Camera()
    c2.add_rotate(0.01, 0.0)
    assert np.array_equal(rtamd.params_to_array(c2.params(m, 64, 48)), single)


def _run_tool(tmp_path, w, h, depth, frames, dx, dy, flags, extra=()):
    r = subprocess.run([TOOL, "--scene", "cornell", "--width", str(w), "--height", str(h), "--depth", str(depth),
                        "--frames", str(frames), "--drag", str(dx), str(dy), "--ppm-dir", str(tmp_path),
                        "--ppm-every", "2", "--bvh-cache", str(tmp_path / "bvh.cache"), "--flags", str(flags),
                        *extra], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    summary = json.loads(r.stdout.strip().splitlines()[-1])
    assert summary["frames"] == frames and summary["fps"] > 0
    return summary


def _orbit_params(m, w, h, frames, dx, dy):
    """The tool's camera per frame (rtamd.Camera = Camera.cpp + updateCamera)."""
    import rtamd
    cam = rtamd.Camera()
    out = []
    for f in range(frames):
        if f > 0:
            cam.add_rotate(dx * 0.25 / 100.0, dy * 0.25 / 100.0)
        out.append(rtamd.params_to_array(cam.params(m, w, h)))
    return out


def _rgb(px, w, h):
    px = px.reshape(h, w)
    return np.stack([px & 0xFF, (px >> 8) & 0xFF, (px >> 16) & 0xFF], -1).astype(np.uint8)


@pytest.mark.gpu
def test_frames_match_the_oracle(tmp_path):
    """Frames of the orbiting camera, rendered by the tool in S_strict arithmetic
    (--flags 64), equal the CPU oracle's frames for the same camera."""
    import rtamd
    from oracle import oracle
    w, h, depth, frames, dx, dy = 96, 64, 3, 5, 7.0, -3.0
    _run_tool(tmp_path, w, h, depth, frames, dx, dy, rtamd.RT_FLAG_STRICT_MATH)
    m = rtamd.Mesh.cornell()
    scene = rtamd.Scene.from_mesh(m, m.build_sbvh())
    for f, p in enumerate(_orbit_params(m, w, h, frames, dx, dy)):
        if f % 2:
            continue
        ref = oracle.render(scene, p, w, h, depth=depth, aux=False)["out"]
        assert np.array_equal(_read_ppm(tmp_path / f"frame_{f:05d}.ppm"), _rgb(ref, w, h)), f"frame {f}"


@pytest.mark.gpu
def test_frames_match_the_render_abi(tmp_path):
    """Default arithmetic (S_ref): the tool's frames equal rt_render's for the same camera;
    a second run reuses the BVH cache."""
    import rtamd
    w, h, depth, frames, dx, dy = 96, 64, 3, 5, 7.0, -3.0
    _run_tool(tmp_path, w, h, depth, frames, dx, dy, 0)
    m = rtamd.Mesh.cornell()
    scene = rtamd.Scene.from_mesh(m, m.build_sbvh())
    ren = rtamd.Renderer(0)
    ren.upload(scene)
    for f, p in enumerate(_orbit_params(m, w, h, frames, dx, dy)):
        if f % 2:
            continue
        ren.set_params(p)
        px = ren.render(w, h, depth=depth)
        assert np.array_equal(_read_ppm(tmp_path / f"frame_{f:05d}.ppm"), _rgb(px, w, h)), f"frame {f}"
    ren.close()
    r2 = subprocess.run([TOOL, "--scene", "cornell", "--width", str(w), "--height", str(h), "--frames", "2",
                         "--bvh-cache", str(tmp_path / "bvh.cache")], capture_output=True, text=True, timeout=300)
    assert r2.returncode == 0 and json.loads(r2.stdout.strip().splitlines()[-1])["bvh_cached"] is True


@pytest.mark.gpu
@pytest.mark.parametrize("depth", [1, 3])
def test_multi_context_frames_match_the_render_abi(tmp_path, depth):
    """--devices 0,0,0: three contexts (device 0 repeated on the one-GPU box) render every frame
    through rt_render_tiled; the frames equal rt_render's for the same orbiting camera."""
    import rtamd
    w, h, frames, dx, dy = 160, 120, 5, 7.0, -3.0
    summary = _run_tool(tmp_path, w, h, depth, frames, dx, dy, 0, extra=("--devices", "0,0,0"))
    assert summary["contexts"] == 3
    m = rtamd.Mesh.cornell()
    ren = rtamd.Renderer(0)
    ren.upload(rtamd.Scene.from_mesh(m, m.build_sbvh()))
    for f, p in enumerate(_orbit_params(m, w, h, frames, dx, dy)):
        if f % 2:
            continue
        ren.set_params(p)
        assert np.array_equal(_read_ppm(tmp_path / f"frame_{f:05d}.ppm"), _rgb(ren.render(w, h, depth=depth), w, h)), f
    ren.close()


@pytest.mark.gpu
@pytest.mark.parametrize("depth,batch", [(1, 4), (3, 3)])
def test_batched_frames_match_the_render_abi(tmp_path, depth, batch):
    """--batch K: the orbit's next K cameras in one rt_render_batch call (K frames in one launch;
    depth 3 in the wavefront mode); every frame equals rt_render's for its camera, including the
    last, part-filled call (7 frames)."""
    import rtamd
    w, h, frames, dx, dy = 160, 120, 7, 7.0, -3.0
    summary = _run_tool(tmp_path, w, h, depth, frames, dx, dy, 0, extra=("--batch", str(batch)))
    assert summary["frames_per_call"] == batch
    m = rtamd.Mesh.cornell()
    ren = rtamd.Renderer(0)
    ren.upload(rtamd.Scene.from_mesh(m, m.build_sbvh()))
    cams = _orbit_params(m, w, h, frames, dx, dy)
    for f, p in enumerate(cams):
        if f % 2:
            continue
        ren.set_params(p)
        assert np.array_equal(_read_ppm(tmp_path / f"frame_{f:05d}.ppm"), _rgb(ren.render(w, h, depth=depth), w, h)), f
    # rt_render_batch through ctypes, into pageable and pinned memory
    import torch
    flags = rtamd.RT_FLAG_WAVEFRONT if depth > 1 else 0
    got = ren.render_batch(w, h, depth, flags, cams[:batch])
    pin = torch.zeros(batch * w * h, dtype=torch.int32, pin_memory=True)
    ren.render_batch(w, h, depth, flags, cams[:batch], out_ptr=pin.data_ptr())
    for i in range(batch):
        ren.set_params(cams[i])
        want = ren.render(w, h, depth=depth)
        assert np.array_equal(got[i], want), i
        assert np.array_equal(pin.numpy().view(np.uint32)[i * w * h:(i + 1) * w * h], want), i
    ren.close()
