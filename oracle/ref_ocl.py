"""Run the reference OpenCL kernel (compiled by oracle/Makefile.ref into
oracle/_ref/) on the GPU.  TEST INFRASTRUCTURE ONLY: used to pin the oracle
(tests/golden/make_golden.py, tests/test_reference_pin_gpu.py,
tests/test_fullsize_gpu.py)."""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF_DIR = os.path.join(HERE, "_ref")
RUNNER = os.path.join(REF_DIR, "libref_ocl.so")
VARIANTS = {"strict": os.path.join(REF_DIR, "volumeRender_strict.hsaco"),
            "default": os.path.join(REF_DIR, "volumeRender_default.hsaco")}

_lib = None


def available() -> bool:
    return os.path.exists(RUNNER) and all(os.path.exists(p) for p in VARIANTS.values())


def lib():
    global _lib
    if _lib is None:
        L = C.CDLL(RUNNER)
        vp = C.c_void_p
        L.refocl_render.restype = C.c_int
        L.refocl_render.argtypes = [C.c_char_p, vp, vp, C.c_int, vp, C.c_int, vp, C.c_int, vp, C.c_int, vp, C.c_int,
                                    vp, vp, C.c_int, vp, C.c_uint32, C.c_uint32, vp, C.c_char_p, C.c_int]
        L.refocl_device_count.restype = C.c_int
        _lib = L
    return _lib


def device_count() -> int:
    return lib().refocl_device_count()


def render(scene, params, w: int, h: int, variant: str = "strict") -> np.ndarray:
    g = (lambda k: scene[k]) if isinstance(scene, dict) else (lambda k: getattr(scene, k))
    a = {k: np.ascontiguousarray(g(k)) for k in ("vertices", "indices", "nodes", "tri_indices", "normals",
                                                  "normals_indices", "materials", "tri_to_material")}
    par = np.ascontiguousarray(params, np.float32).reshape(32)
    out = np.zeros(w * h, np.uint32)
    eb = C.create_string_buffer(512)

    def p(x):
        return x.ctypes.data_as(C.c_void_p)
    rc = lib().refocl_render(VARIANTS[variant].encode(), p(par), p(a["vertices"]), a["vertices"].shape[0],
                             p(a["indices"]), a["indices"].size, p(a["nodes"]), a["nodes"].shape[0],
                             p(a["tri_indices"]), a["tri_indices"].size, p(a["normals"]), a["normals"].shape[0],
                             p(a["normals_indices"]), p(a["materials"]), a["materials"].shape[0],
                             p(a["tri_to_material"]), w, h, p(out), eb, 512)
    if rc != 0:
        raise RuntimeError(f"reference OpenCL run failed: {eb.value.decode()}")
    return out


KEYS = ("vertices", "indices", "nodes", "tri_indices", "normals", "normals_indices", "materials", "tri_to_material")


def render_subprocess(scene, params, w: int, h: int, variant: str, workdir: str, timeout: int = 300) -> np.ndarray:
    """Run the reference kernel in a child process (the OpenCL runtime must not share a
    process with torch's HIP runtime): the scene arrays go through an uncompressed .npz
    in `workdir`, the frame comes back as a .npy."""
    import subprocess
    import sys
    g = (lambda k: scene[k]) if isinstance(scene, dict) else (lambda k: getattr(scene, k))
    src = os.path.join(workdir, "ref_scene.npz")
    dst = os.path.join(workdir, "ref_out.npy")
    np.savez(src, params=np.asarray(params, np.float32).reshape(32), w=w, h=h,
             **{k: np.ascontiguousarray(g(k)) for k in KEYS})
    root = os.path.dirname(HERE)
    code = ("import sys; sys.path.insert(0, %r); from oracle import ref_ocl; ref_ocl._child(%r, %r, %r)"
            % (root, src, dst, variant))
    res = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=timeout)
    if res.returncode != 0:
        raise RuntimeError(f"reference kernel run failed: {res.stderr[-2000:]}")
    out = np.load(dst)
    os.remove(src)
    os.remove(dst)
    return out


def _child(src: str, dst: str, variant: str) -> None:
    d = dict(np.load(src))
    np.save(dst, render(d, d["params"], int(d["w"]), int(d["h"]), variant))
