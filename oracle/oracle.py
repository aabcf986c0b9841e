"""ctypes wrapper of the CPU oracle (oracle/rt_oracle.c).

TEST INFRASTRUCTURE ONLY -- imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product package.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "liboracle.so")


class ostats(C.Structure):
    _fields_ = [("rays", C.c_uint64 * 3), ("inner", C.c_uint64 * 3), ("leaf", C.c_uint64 * 3),
                ("tris", C.c_uint64 * 3), ("max_stack", C.c_uint64), ("stack_overflow", C.c_uint64)]

    def as_dict(self):
        kinds = ("primary", "shadow", "secondary")
        d = {}
        for i, k in enumerate(kinds):
            d[k] = {"rays": int(self.rays[i]), "inner": int(self.inner[i]), "leaf": int(self.leaf[i]),
                    "tris": int(self.tris[i])}
        d["max_stack"] = int(self.max_stack)
        d["stack_overflow"] = int(self.stack_overflow)
        return d


_lib = None


def build():
    subprocess.run(["make", "-C", HERE], check=True, capture_output=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        vp = C.c_void_p
        L.oracle_render.restype = C.c_int
        L.oracle_render.argtypes = [vp, vp, vp, vp, C.c_int32, vp, C.c_int32, vp, vp, vp, vp, C.c_uint32,
                                    C.c_uint32, C.c_int, C.c_uint32, C.c_int64, C.c_int64, C.c_int64, vp, vp, vp,
                                    vp, C.POINTER(ostats), C.c_int]
        L.oracle_normalize.argtypes = [vp, vp]
        L.oracle_ray_tri.restype = C.c_float
        L.oracle_ray_tri.argtypes = [vp, vp, vp, vp, vp]
        L.oracle_rgb_to_int.restype = C.c_uint32
        L.oracle_rgb_to_int.argtypes = [C.c_float, C.c_float, C.c_float]
        L.sbvh_oracle_build.restype = C.c_int
        L.sbvh_oracle_build.argtypes = [vp, C.c_int32, vp, C.c_int32, C.POINTER(vp), C.POINTER(C.c_int32),
                                        C.POINTER(C.POINTER(C.c_int32)), C.POINTER(C.c_int32)]
        L.sbvh_oracle_free.argtypes = [vp]
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def render(scene, params, w, h, depth=3, flags=0, pixels=None, nthreads=None, aux=True):
    """Render with the oracle.

    scene  : object with numpy arrays vertices, indices, nodes, tri_indices, normals,
             normals_indices, materials, tri_to_material (rtamd.Scene or a fixture dict)
    params : float32[32] Params block
    pixels : None (whole frame) or (start, count, stride) over linear pixel index y*w+x
    Returns dict(out, hits, t, rgb, stats).
    """
    g = (lambda k: scene[k]) if isinstance(scene, dict) else (lambda k: getattr(scene, k))
    arr = {k: np.ascontiguousarray(g(k)) for k in ("vertices", "indices", "nodes", "tri_indices", "normals",
                                                    "normals_indices", "materials", "tri_to_material")}
    par = np.ascontiguousarray(params, dtype=np.float32).reshape(32)
    if pixels is None:
        pixels = (0, w * h, 1)
    p0, n, st = (int(v) for v in pixels)
    d = max(depth, 1)
    out = np.zeros(n, np.uint32)
    hits = np.zeros((n, d, 2), np.int32) if aux else None
    tv = np.zeros((n, d), np.float32) if aux else None
    rgb = np.zeros((n, 3), np.float32) if aux else None
    stats = ostats()
    if nthreads is None:
        nthreads = min(os.cpu_count() or 1, 16)
    rc = lib().oracle_render(_p(par), _p(arr["vertices"]), _p(arr["indices"]), _p(arr["nodes"]),
                             arr["nodes"].shape[0], _p(arr["tri_indices"]), arr["tri_indices"].size,
                             _p(arr["normals"]), _p(arr["normals_indices"]), _p(arr["materials"]),
                             _p(arr["tri_to_material"]), w, h, depth, flags, p0, n, st, _p(out), _p(hits), _p(tv),
                             _p(rgb), C.byref(stats), nthreads)
    if rc != 0:
        raise RuntimeError(f"oracle_render failed: {rc}")
    res = {"out": out, "stats": stats.as_dict()}
    if aux:
        res.update(hits=hits[:, :depth], t=tv[:, :depth], rgb=rgb)
    return res


def sbvh(vertices, indices):
    """The reference's SplitBVHBuilder + BVH_Cuda::build_from_bvh2 restated (sbvh_oracle.c).
    vertices: float32 [nv, 4]; indices: int32 [3 * ntri].  Returns (nodes [nn, 12] float32 view of
    BVH_Node_ records, tri_indices int32 (= 3 * triangle))."""
    L = lib()
    v = np.ascontiguousarray(vertices, np.float32).reshape(-1, 4)
    ix = np.ascontiguousarray(indices, np.int32).reshape(-1)
    nodes_p, refs_p = C.c_void_p(), C.POINTER(C.c_int32)()
    nn, nr = C.c_int32(), C.c_int32()
    rc = L.sbvh_oracle_build(_p(v), v.shape[0], _p(ix), ix.size // 3, C.byref(nodes_p), C.byref(nn),
                             C.byref(refs_p), C.byref(nr))
    if rc != 0:
        raise RuntimeError("sbvh_oracle_build failed")
    nodes = np.ctypeslib.as_array(C.cast(nodes_p, C.POINTER(C.c_float)), (max(nn.value, 1) * 12,)).copy()
    refs = np.ctypeslib.as_array(refs_p, (max(nr.value, 1),)).copy()[:nr.value]
    L.sbvh_oracle_free(nodes_p)
    L.sbvh_oracle_free(C.cast(refs_p, C.c_void_p))
    return nodes.reshape(-1, 12)[:nn.value], refs


def bytes_per_ray(stats: dict, kind: str) -> float:
    """Algorithmic bytes per traced ray: 80*inner + 16*leaf + 64*tri."""
    s = stats[kind]
    if s["rays"] == 0:
        return 0.0
    return (80.0 * s["inner"] + 16.0 * s["leaf"] + 64.0 * s["tris"]) / s["rays"]
