"""The synthetic scenes and frames of BASELINE.json's configs, shared by
bench.py and the full-size parity tests.

C1: the 12-triangle Cornell room at 256x256, depth 1 (the reference's CPU-path config).
C2: a 70,144-tri torus knot at 1080p, primary rays only.
C3: a 1M-tri value-noise heightfield at 1080p, primary + 1 shadow ray (the metric's config).
C4: the C3 scene at 4K (the multi-GPU scaling curve).
C5: 10 x C3 on a 5x2 grid = 10M tris at 1080p, depth 3, wavefront mode with per-bounce ray
    sorting (c5u: unsorted, for A/B).
"""
from __future__ import annotations

import os
import tempfile
import time

# C3 terrain extent: fills the default camera's 1080p view (Camera.cpp:6-19)
HF_EXT = (-150.0, 650.0, -150.0, 650.0)

RT_FLAG_NO_SHADOW = 1
RT_FLAG_WAVEFRONT = 8
RT_FLAG_WF_SORT = 32

CONFIGS = {
    # BASELINE.json configs[0]: the reference's CPU-path case, here on the GPU path
    "c1": dict(scene="cornell", w=256, h=256, depth=1, flags=0,
               desc="C1: 12-tri Cornell room (10 wall + 2 quad tris), 256x256, primary + 1 shadow ray"),
    # configs[1]: ~70k-tri mesh, primary only
    "c2": dict(scene="knot", nu=256, nv=137, w=1920, h=1080, depth=1, flags=RT_FLAG_NO_SHADOW,
               desc="C2: 70,144-tri torus knot, 1920x1080, primary rays only"),
    # configs[2] -- the metric's configuration
    "c3": dict(scene="heightfield", nx=500, nz=1000, amp=10.0, seed=0x5EED, ext=HF_EXT, w=1920, h=1080, depth=1,
               flags=0,
               desc="C3: 1M-tri value-noise heightfield (500x1000 cells x2, seed 0x5EED), 1920x1080, "
                    "primary + 1 shadow ray"),
    # configs[3]: C3 scene at 4K (multi-GPU scaling curve)
    "c4": dict(scene="heightfield", nx=500, nz=1000, amp=10.0, seed=0x5EED, ext=HF_EXT, w=3840, h=2160, depth=1,
               flags=0, desc="C4: C3 scene at 3840x2160, primary + 1 shadow ray"),
    # configs[4]: 10M tris (10 x C3 on a 5x2 grid), depth 3 (primary + 2 bounces, shadows), in
    # the wavefront mode with per-bounce ray sorting: each bounce queue is reordered within
    # screen-local chunks of 1024 rays by the rays' direction along the scene's thinnest axis
    # (rt_render.hip wf_local_sort_kernel)
    "c5": dict(scene="hf10", nx=500, nz=1000, amp=10.0, seed=0x5EED, ext=(-80.0, 80.0, -200.0, 200.0), w=1920,
               h=1080, depth=3, flags=RT_FLAG_WAVEFRONT | RT_FLAG_WF_SORT,
               dae=False,  # a 1 GB Collada text file is not worth the round trip; built in memory
               desc="C5: 10M-tri merged scene (10 x C3 on a 5x2 grid), 1920x1080, 3 bounces with shadows, "
                    "wavefront mode with per-bounce ray sorting (screen-local chunks, by direction)"),
    # A/B: the same without the sort (queues in the compaction's tile order)
    "c5u": dict(scene="hf10", nx=500, nz=1000, amp=10.0, seed=0x5EED, ext=(-80.0, 80.0, -200.0, 200.0), w=1920,
                h=1080, depth=3, flags=RT_FLAG_WAVEFRONT, dae=False,
                desc="C5 scene and frame, wavefront mode, bounce queues unsorted (tile order)"),
}


def make_mesh(cfg, via_dae=True):
    """The config's synthetic mesh; with via_dae (configs C2-C4) it is written
    as the reference-subset Collada file and read back through the ColladaLoader path
    (rt_mesh_save_dae / rt_mesh_load_dae), as the reference application loads its scene."""
    import rtamd
    if cfg["scene"] == "heightfield":
        mesh = rtamd.Mesh.heightfield(cfg["nx"], cfg["nz"], cfg["amp"], cfg["seed"], cfg["ext"])
    elif cfg["scene"] == "knot":
        mesh = rtamd.Mesh.torus_knot(cfg["nu"], cfg["nv"])
    elif cfg["scene"] == "cornell":
        mesh = rtamd.Mesh.cornell()
    elif cfg["scene"] == "hf10":
        tile = rtamd.Mesh.heightfield(cfg["nx"], cfg["nz"], cfg["amp"], cfg["seed"], cfg["ext"])
        mesh = rtamd.Mesh()
        mesh.append_grid(tile, 5, 2, 160.0, 400.0, 1.0)
    else:
        raise ValueError(cfg["scene"])
    if via_dae and cfg.get("dae", True):
        with tempfile.TemporaryDirectory() as td:
            path = os.path.join(td, "scene.dae")
            mesh.save_dae(path)
            mesh = rtamd.Mesh.load_dae(path)
    return mesh


def make_scene(cfg, threads=0, builder="sbvh", via_dae=True):
    """(mesh, bvh, build seconds): the config's mesh and its BVH (the reference's
    SplitBVHBuilder restated, same bytes; or binned SAH for A/B)."""
    mesh = make_mesh(cfg, via_dae)
    t0 = time.time()
    bvh = mesh.build_sbvh(threads) if builder == "sbvh" else mesh.build_bvh(8, threads)
    return mesh, bvh, time.time() - t0
