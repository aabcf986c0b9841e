"""Generate the golden fixtures that pin the oracle to the reference kernel.

Two phases:

  python tests/golden/make_golden.py inputs      (this container, CPU)
      builds each fixture's inputs -- the raytracer_bvh array arguments and the
      Params block -- with this repo's host tools (and the reference's own
      cubes2.obj / sphere.obj assets when /root/reference is present) and writes
      tests/golden/<name>.npz.

  python tests/golden/make_golden.py reference   (GPU box, MI355X)
      runs the REFERENCE kernel, compiled from x64/Release/volumeRender.cl by
      oracle/Makefile.ref (strict and default variants), on every fixture's
      inputs through the ROCm OpenCL runtime (oracle/ref_ocl.py) and writes
      gpurun_out/golden/<name>.ref.npz with its packed BGR output, which is then
      merged into tests/golden/<name>.npz (keys ref_strict, ref_default).

The reference kernel always runs RAY_TRACE_DEPTH = 3 bounces with shadows
(volumeRender.cl:12), so every fixture is depth 3.  Widths and heights are
multiples of 8: the reference's padded NDRange aliases x >= w threads into the
next row otherwise.
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "real-time-opencl-raytracer_amd"))
sys.path.insert(0, ROOT)

REF_DATA = "/root/reference/x64/Release/data"
DEPTH = 3


def _scene_dict(mesh, bvh, w, h, **cam):
    import rtamd
    s = rtamd.Scene.from_mesh(mesh, bvh).arrays()
    s["params"] = rtamd.params_to_array(mesh.camera_params(w, h, **cam))
    s["w"] = np.int32(w)
    s["h"] = np.int32(h)
    s["depth"] = np.int32(DEPTH)
    return s


def _overflow_scene():
    """A comb BVH 70 levels deep where every level pushes: the 65-entry stack
    overflows (volumeRender.cl:914) and traversal returns -1 (a miss)."""
    import rtamd
    m = rtamd.Mesh.random(80, extent=40.0, size=8.0, seed=7)
    a = m.arrays()
    ntri = a["indices"].size // 3
    depth = 70
    lo = np.append(a["scene_min"], 1.0).astype(np.float32)
    hi = np.append(a["scene_max"], 1.0).astype(np.float32)
    nodes = []
    refs = []
    # pre-order: inner(k) -> left = inner(k+1), right = leaf(k)
    def node(minv, maxv, l, r, off, cnt):
        rec = np.zeros(12, np.float32)
        rec[0:4] = minv
        rec[4:8] = maxv
        rec[8:12] = np.array([l, r, off, cnt], np.int32).view(np.float32)
        return rec
    # layout: index 2k = inner k, 2k+1 = leaf k (left subtree first means the
    # inner chain precedes the leaves in strict pre-order; the kernel does not
    # care about ordering, only about the indices).
    for k in range(depth):
        inner = 2 * k
        leaf = 2 * k + 1
        nxt = 2 * (k + 1) if k + 1 < depth else 2 * k + 1
        nodes.append(node(lo, hi, nxt, leaf, -1, 0))
        t = k % ntri
        nodes.append(node(lo, hi, -1, -1, len(refs), 1))
        refs.append(3 * t)
    nodes = np.stack(nodes).astype(np.float32)
    d = {k: a[k] for k in ("vertices", "indices", "normals", "normals_indices", "materials", "tri_to_material",
                           "scene_min", "scene_max")}
    d["nodes"] = nodes
    d["tri_indices"] = np.array(refs, np.int32)
    d["params"] = rtamd.params_to_array(m.camera_params(64, 64))
    d["w"], d["h"], d["depth"] = np.int32(64), np.int32(64), np.int32(DEPTH)
    return d


def _bad_node_scene():
    """Cornell BVH with one inner node's right child set to -1: the reference
    returns -1 whenever traversal pops that node (volumeRender.cl:841)."""
    import rtamd
    m = rtamd.Mesh.torus_knot(48, 24)
    b = m.build_bvh()
    d = _scene_dict(m, b, 96, 96)
    ni = d["nodes"].view(np.int32).reshape(-1, 12)
    inner = np.nonzero(ni[:, 8] >= 0)[0]
    victim = inner[len(inner) // 3]
    ni[victim, 9] = -1
    return d


def fixtures():
    import rtamd
    fx = {}
    m = rtamd.Mesh.cornell()
    b = m.build_bvh()
    fx["cornell12"] = _scene_dict(m, b, 256, 256)
    fx["cornell12_orbit"] = _scene_dict(m, b, 128, 96, extra_alpha=0.7, extra_beta=-0.3)
    m = rtamd.Mesh.torus_knot(128, 64)
    fx["knot16k"] = _scene_dict(m, m.build_bvh(), 256, 256)
    m = rtamd.Mesh.heightfield(100, 200, 10.0, 0x5EED)
    fx["hf40k"] = _scene_dict(m, m.build_bvh(), 256, 256)
    m = rtamd.Mesh.random(2000, 80.0, 6.0, 1)
    fx["rand2k"] = _scene_dict(m, m.build_bvh(), 128, 128)
    m = rtamd.Mesh.random(3000, 60.0, 10.0, 3)
    fx["rand3k_bigleaf"] = _scene_dict(m, m.build_bvh(max_leaf=64), 128, 128)
    one = rtamd.Mesh.from_arrays(np.array([[-50, -20, 0, 1], [50, -20, 0, 1], [0, 60, 10, 1]], np.float32),
                                 np.array([0, 1, 2], np.int32))
    fx["single_tri_rootleaf"] = _scene_dict(one, one.build_bvh(), 64, 64)
    fx["overflow_comb"] = _overflow_scene()
    fx["bad_node"] = _bad_node_scene()
    m = rtamd.Mesh.random(4000, 100.0, 12.0, 3)   # long triangles: spatial splits, duplicated refs
    fx["rand4k_sbvh"] = _scene_dict(m, m.build_sbvh(), 128, 128)
    if os.path.isdir(REF_DATA):
        # the reference application's own scene: data/collada/cubes2.DAE through the
        # Collada path and the spatial-split BVH (RayTracer.cpp's startup)
        m = rtamd.Mesh.load_dae(os.path.join(REF_DATA, "collada", "cubes2.DAE"))
        fx["cubes2_dae"] = _scene_dict(m, m.build_sbvh(), 256, 192)
        m = rtamd.Mesh.load_obj(os.path.join(REF_DATA, "models", "cubes2.obj"))
        fx["cubes2_obj"] = _scene_dict(m, m.build_bvh(), 256, 192)
        m = rtamd.Mesh.load_obj(os.path.join(REF_DATA, "sphere.obj"))
        fx["sphere_obj"] = _scene_dict(m, m.build_bvh(), 128, 128, radius=5.0)
    return fx


def main(phase: str, only=()):
    if phase == "inputs":
        for name, d in fixtures().items():
            if only and name not in only:
                continue
            np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **d)
            print("wrote", name, int(d["indices"].size // 3), "tris", int(d["w"]), "x", int(d["h"]))
    elif phase == "reference":
        from oracle import ref_ocl
        outdir = os.path.join(ROOT, "gpurun_out", "golden")
        os.makedirs(outdir, exist_ok=True)
        print("OpenCL GPU devices:", ref_ocl.device_count())
        for fn in sorted(os.listdir(HERE)):
            if not fn.endswith(".npz") or fn.endswith(".ref.npz"):
                continue
            if only and fn[:-4] not in only:
                continue
            d = dict(np.load(os.path.join(HERE, fn)))
            w, h = int(d["w"]), int(d["h"])
            res = {}
            for var in ("strict", "default"):
                res[f"ref_{var}"] = ref_ocl.render(d, d["params"], w, h, var)
            np.savez_compressed(os.path.join(outdir, fn.replace(".npz", ".ref.npz")), **res)
            print("reference ran", fn, {k: int(np.count_nonzero(v)) for k, v in res.items()})
    elif phase == "merge":
        src = os.path.join(ROOT, "gpurun_out", "golden")
        for fn in sorted(os.listdir(src)):
            name = fn.replace(".ref.npz", ".npz")
            d = dict(np.load(os.path.join(HERE, name)))
            d.update(dict(np.load(os.path.join(src, fn))))
            np.savez_compressed(os.path.join(HERE, name), **d)
            print("merged", name)
    else:
        raise SystemExit("usage: make_golden.py inputs|reference|merge [fixture ...]")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "inputs", tuple(sys.argv[2:]))
