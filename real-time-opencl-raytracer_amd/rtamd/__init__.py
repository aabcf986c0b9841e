"""rtamd -- Python host mirror of the MI355X render path (ctypes over librtamd.so).

The reference drives its kernel from C++ (RayTracer.cpp: initRayTrace :858,
initCLVolume2 :1234, updateCamera :609, raytrace_gpgpu :330).  This module is
the same sequence over the C ABI in include/rt_abi.h and include/rt_host.h:

    mesh  = Mesh.heightfield(500, 1000, 10.0, 0x5EED)     # Mesh::init
    bvh   = mesh.build_bvh()                              # BVH2::setMesh + BVH_Cuda::build_from_bvh2
    scene = Scene.from_mesh(mesh, bvh)                    # the kernel's array arguments
    r     = Renderer(device=0); r.upload(scene)           # clCreateBuffer x9 + clSetKernelArg
    r.set_params(mesh.camera_params(1920, 1080))          # updateCamera
    img   = r.render(1920, 1080, depth=1)                 # raytrace_gpgpu

There is no CPU fallback: if librtamd.so is missing or no GPU is present the
render calls raise.  The CPU restatement under oracle/ is test infrastructure.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass, field
from typing import Optional

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(_HERE)
LIB_PATH = os.environ.get("RTAMD_LIB") or os.path.join(PKG_ROOT, "lib", "librtamd.so")

RT_FLAG_NO_SHADOW = 1
RT_FLAG_HW_MATH = 2
RT_FLAG_EXACT_DIV = 4
RT_FLAG_STATIC_ORDER = 16
RT_FLAG_WAVEFRONT = 8
RT_FLAG_WF_SORT = 32
RT_FLAG_STRICT_MATH = 64
RT_MAX_DEPTH = 8
RT_MAX_BATCH = int(os.environ.get("RTAMD_MAX_BATCH", "8"))   # rt_render_device_batch frames per launch (RTAMD_MAX_BATCH: an A/B build's)
ERRORS = {0: "RT_OK", -1: "RT_ERR_INVALID_ARG", -2: "RT_ERR_DEVICE", -3: "RT_ERR_NO_SCENE",
          -4: "RT_ERR_OUT_OF_MEMORY", -5: "RT_ERR_BAD_SCENE"}


class RtError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{ERRORS.get(code, code)}: {msg}")
        self.code = code


class rt_float4(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("z", C.c_float), ("w", C.c_float)]


class rt_params(C.Structure):
    _fields_ = [(n, rt_float4) for n in
                ("a", "b", "c", "campos", "light_pos", "light_color", "scene_aabb_min", "scene_aabb_max")]


class rt_aux(C.Structure):
    _fields_ = [("hits", C.c_void_p), ("t", C.c_void_p), ("rgb", C.c_void_p)]


class rt_tiling(C.Structure):
    _fields_ = [("rank", C.c_int32), ("nranks", C.c_int32), ("band_rows", C.c_int32), ("reserved", C.c_int32)]


class rt_mesh_view(C.Structure):
    _fields_ = [("vertices", C.c_void_p), ("num_vertices", C.c_int32),
                ("indices", C.c_void_p), ("num_indices", C.c_int32),
                ("normals", C.c_void_p), ("num_normals", C.c_int32),
                ("normals_indices", C.c_void_p),
                ("materials", C.c_void_p), ("num_materials", C.c_int32),
                ("tri_to_material", C.c_void_p),
                ("scene_min", C.c_float * 3), ("scene_max", C.c_float * 3)]


class rt_bvh_view(C.Structure):
    _fields_ = [("nodes", C.c_void_p), ("num_nodes", C.c_int32),
                ("tri_indices", C.c_void_p), ("num_tri_indices", C.c_int32),
                ("max_depth", C.c_int32), ("num_leaves", C.c_int32),
                ("build_seconds", C.c_double)]


# every symbol include/rt_abi.h and include/rt_host.h declare
ABI_SYMBOLS = ["rt_create", "rt_upload_scene", "rt_set_params", "rt_render", "rt_render_tiled", "rt_tiled_direct_ok",
               "rt_last_enqueue_time", "rt_scene_copy",
               "rt_render_device", "rt_render_device_batch", "rt_render_batch",
               "rt_tiling_pixels", "rt_assemble_bands", "rt_assemble_bands_batch", "rt_comm_unique_id", "rt_comm_create", "rt_comm_destroy",
               "rt_comm_last_error", "rt_frame_gather", "rt_frame_exchange", "rt_frame_slot_wait",
               "rt_frame_ready_wait", "rt_ipc_export", "rt_ipc_open", "rt_ipc_close", "rt_bands_put",
               "rt_peer_access", "rt_frame_sync_words", "rt_bands_put_sync", "rt_frame_present", "rt_frame_release",
               "rt_frame_sync_status", "rt_frame_checksum", "rt_shared_alloc", "rt_shared_free", "rt_copy_device",
               "rt_scene_image_size", "rt_scene_image_pack",
               "rt_scene_image_load", "rt_fetch_counts", "rt_gather_peak", "rt_chase_peak", "rt_chase_latency", "rt_wave_timeline", "rt_last_timing", "rt_timing_average", "rt_last_deferred", "rt_overflow_count", "rt_destroy", "rt_last_error",
               "rt_abi_version"]
HOST_SYMBOLS = ["rt_mesh_create", "rt_mesh_destroy", "rt_mesh_view_get", "rt_mesh_set", "rt_mesh_load_obj",
                "rt_mesh_load_dae", "rt_mesh_save_dae",
                "rt_mesh_gen_cornell", "rt_mesh_gen_torus_knot", "rt_mesh_gen_heightfield", "rt_mesh_gen_random",
                "rt_mesh_append_grid", "rt_bvh_build", "rt_bvh_build_sbvh", "rt_bvh_view_get", "rt_bvh_destroy", "rt_bvh_save",
                "rt_bvh_load", "rt_camera_params", "rt_camera_create", "rt_camera_destroy", "rt_camera_add_rotate",
                "rt_camera_add_radius", "rt_camera_frame_params"]

_lib = None


def lib() -> C.CDLL:
    """Load librtamd.so (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RtError(-2, f"{LIB_PATH} not built (run __graft_entry__.build() or make -C {PKG_ROOT})")
        # torch bundles its own libamdhip64.so.7 / libhsa-runtime64.so.1 (same SONAMEs as
        # /opt/rocm's).  Let torch load them first so the process has ONE HIP runtime that
        # both torch tensors (device memory, streams, RCCL) and librtamd.so use.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = C.CDLL(LIB_PATH)
        vp, i32, u32, f32 = C.c_void_p, C.c_int32, C.c_uint32, C.c_float
        sig = {
            "rt_create": (C.c_int, [C.c_int, C.POINTER(vp)]),
            "rt_upload_scene": (C.c_int, [vp, vp, i32, vp, i32, vp, i32, vp, i32, vp, i32, vp, vp, i32, vp]),
            "rt_set_params": (C.c_int, [vp, C.POINTER(rt_params)]),
            "rt_render": (C.c_int, [vp, u32, u32, i32, u32, vp, C.POINTER(rt_aux)]),
            "rt_render_tiled": (C.c_int, [C.POINTER(vp), i32, u32, u32, i32, u32, vp]),
            "rt_scene_copy": (C.c_int, [vp, vp]),
            "rt_tiled_direct_ok": (C.c_int32, [i32, C.POINTER(C.c_uint64)]),
            "rt_last_enqueue_time": (C.c_int, [vp, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
            "rt_render_device": (C.c_int, [vp, u32, u32, i32, u32, C.POINTER(rt_tiling), vp, C.POINTER(rt_aux), vp]),
            "rt_render_device_batch": (C.c_int, [vp, u32, u32, i32, u32, C.POINTER(rt_tiling), C.POINTER(rt_params), i32,
                                                 vp, C.c_uint64, vp]),
            "rt_render_batch": (C.c_int, [vp, u32, u32, i32, u32, C.POINTER(rt_params), i32, vp]),
            "rt_tiling_pixels": (C.c_int64, [u32, u32, C.POINTER(rt_tiling)]),
            "rt_assemble_bands": (C.c_int, [vp, vp, C.c_uint64, u32, u32, i32, i32, vp]),
            "rt_assemble_bands_batch": (C.c_int, [vp, vp, C.c_uint64, C.c_uint64, i32, u32, u32, i32, i32, vp]),
            "rt_comm_unique_id": (C.c_int, [vp, i32]),
            "rt_comm_create": (C.c_int, [i32, i32, i32, vp, i32, C.POINTER(vp)]),
            "rt_comm_destroy": (C.c_int, [vp]),
            "rt_comm_last_error": (C.c_char_p, []),
            "rt_frame_gather": (C.c_int, [vp, vp, C.c_uint64, vp, vp, u32, u32, i32, vp]),
            "rt_frame_exchange": (C.c_int, [vp, i32, i32, vp, C.c_uint64, vp, vp, u32, u32, i32, vp]),
            "rt_frame_slot_wait": (C.c_int, [vp, i32, vp]),
            "rt_ipc_export": (C.c_int, [i32, vp, vp, i32, C.POINTER(C.c_uint64)]),
            "rt_ipc_open": (C.c_int, [i32, vp, i32, C.POINTER(vp)]),
            "rt_ipc_close": (C.c_int, [i32, vp]),
            "rt_bands_put": (C.c_int, [vp, vp, u32, u32, vp, vp]),
            "rt_peer_access": (C.c_int, [i32, i32, C.POINTER(i32)]),
            "rt_frame_sync_words": (C.c_int64, [i32, i32]),
            "rt_bands_put_sync": (C.c_int, [vp, vp, u32, u32, vp, vp, vp, i32, i32, u32, u32, vp]),
            "rt_frame_present": (C.c_int, [vp, i32, i32, u32, i32, u32, i32, vp]),
            "rt_frame_release": (C.c_int, [vp, i32, i32, u32, vp]),
            "rt_frame_sync_status": (C.c_int, [vp, C.POINTER(u32), C.POINTER(u32)]),
            "rt_frame_checksum": (C.c_int, [vp, C.c_uint64, vp, vp]),
            "rt_shared_alloc": (C.c_int, [i32, C.c_uint64, C.POINTER(vp)]),
            "rt_shared_free": (C.c_int, [i32, vp]),
            "rt_copy_device": (C.c_int, [vp, vp, C.c_uint64, vp]),
            "rt_frame_ready_wait": (C.c_int, [vp, i32, vp]),
            "rt_scene_image_size": (C.c_int, [vp, C.POINTER(C.c_uint64)]),
            "rt_scene_image_pack": (C.c_int, [vp, vp, C.c_uint64, vp]),
            "rt_scene_image_load": (C.c_int, [vp, vp, C.c_uint64, vp]),
            "rt_fetch_counts": (C.c_int, [vp, u32, u32, i32, u32, C.POINTER(C.c_uint64)]),
            "rt_gather_peak": (C.c_int, [vp, u32, u32, C.POINTER(f32), C.POINTER(C.c_uint64)]),
            "rt_chase_peak": (C.c_int, [vp, u32, u32, u32, C.POINTER(f32), C.POINTER(C.c_uint64)]),
            "rt_chase_latency": (C.c_int, [vp, u32, u32, u32, u32, C.POINTER(f32), C.POINTER(C.c_uint64)]),
            "rt_wave_timeline": (C.c_int, [vp, u32, u32, i32, u32, i32, vp, C.c_uint64, C.POINTER(C.c_uint64)]),
            "rt_last_timing": (C.c_int, [vp, C.POINTER(f32), C.POINTER(f32)]),
            "rt_timing_average": (C.c_int, [vp, i32, C.POINTER(f32), C.POINTER(f32)]),
            "rt_last_deferred": (C.c_int, [vp, C.POINTER(u32)]),
            "rt_overflow_count": (C.c_int, [vp, C.POINTER(C.c_uint64)]),
            "rt_destroy": (C.c_int, [vp]),
            "rt_last_error": (C.c_char_p, [vp]),
            "rt_abi_version": (C.c_int, []),
            "rt_mesh_create": (vp, []),
            "rt_mesh_destroy": (None, [vp]),
            "rt_mesh_view_get": (C.c_int, [vp, C.POINTER(rt_mesh_view)]),
            "rt_mesh_set": (C.c_int, [vp, vp, i32, vp, i32, vp, i32, vp, vp, i32, vp]),
            "rt_mesh_load_obj": (C.c_int, [vp, C.c_char_p]),
            "rt_mesh_gen_cornell": (C.c_int, [vp]),
            "rt_mesh_gen_torus_knot": (C.c_int, [vp, i32, i32]),
            "rt_mesh_gen_heightfield": (C.c_int, [vp, i32, i32, f32, u32, f32, f32, f32, f32]),
            "rt_mesh_gen_random": (C.c_int, [vp, i32, f32, f32, u32]),
            "rt_mesh_append_grid": (C.c_int, [vp, vp, i32, i32, f32, f32, f32]),
            "rt_mesh_load_dae": (C.c_int, [vp, C.c_char_p]),
            "rt_mesh_save_dae": (C.c_int, [vp, C.c_char_p]),
            "rt_bvh_build": (C.c_int, [vp, i32, i32, C.POINTER(vp)]),
            "rt_bvh_build_sbvh": (C.c_int, [vp, i32, C.POINTER(vp)]),
            "rt_bvh_view_get": (C.c_int, [vp, C.POINTER(rt_bvh_view)]),
            "rt_bvh_destroy": (None, [vp]),
            "rt_bvh_save": (C.c_int, [vp, vp, C.c_char_p]),
            "rt_bvh_load": (C.c_int, [vp, C.c_char_p, C.POINTER(vp)]),
            "rt_camera_params": (C.c_int, [vp, u32, u32, f32, f32, f32, vp, vp, C.POINTER(rt_params)]),
            "rt_camera_create": (vp, [f32]),
            "rt_camera_destroy": (None, [vp]),
            "rt_camera_add_rotate": (C.c_int, [vp, f32, f32]),
            "rt_camera_add_radius": (C.c_int, [vp, f32]),
            "rt_camera_frame_params": (C.c_int, [vp, vp, u32, u32, vp, vp, C.POINTER(rt_params)]),
        }
        for name, (res, args) in sig.items():
            if not hasattr(L, name):   # an older build loaded for an A/B (RTAMD_LIB): its own symbols only
                continue
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def library_digest() -> str:
    """sha256 (first 16 hex digits) of the librtamd.so this process loads: ties a profile
    taken in a separate run to the exact kernels it measured."""
    import hashlib
    with open(LIB_PATH, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def _ptr(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def _check(code: int, ctx=None):
    if code != 0:
        msg = lib().rt_last_error(ctx)
        raise RtError(code, msg.decode() if msg else "")


def params_to_array(p: rt_params) -> np.ndarray:
    return np.frombuffer(bytes(p), dtype=np.float32).copy()


def array_to_params(a: np.ndarray) -> rt_params:
    a = np.ascontiguousarray(a, dtype=np.float32).reshape(32)
    return rt_params.from_buffer_copy(a.tobytes())


@dataclass
class Scene:
    """The raytracer_bvh array arguments (volumeRender.cl:1043-1075) as numpy arrays.

    nodes: float32 (nn, 12) raw BVH_Node_ words (words 8..11 are int32 bits)
    materials: float32 (nm, 44) raw Material words (words 0..3 are int32 bits)
    """
    vertices: np.ndarray
    indices: np.ndarray
    nodes: np.ndarray
    tri_indices: np.ndarray
    normals: np.ndarray
    normals_indices: np.ndarray
    materials: np.ndarray
    tri_to_material: np.ndarray
    scene_min: np.ndarray = field(default_factory=lambda: np.zeros(3, np.float32))
    scene_max: np.ndarray = field(default_factory=lambda: np.zeros(3, np.float32))

    @property
    def num_triangles(self) -> int:
        return int(self.indices.size // 3)

    def nodes_int(self) -> np.ndarray:
        return self.nodes.view(np.int32)

    def arrays(self) -> dict:
        return {k: getattr(self, k) for k in ("vertices", "indices", "nodes", "tri_indices", "normals",
                                              "normals_indices", "materials", "tri_to_material",
                                              "scene_min", "scene_max")}

    @staticmethod
    def from_arrays(d) -> "Scene":
        def g(k, dt):
            return np.ascontiguousarray(d[k], dtype=dt)
        return Scene(g("vertices", np.float32).reshape(-1, 4), g("indices", np.int32).reshape(-1),
                     g("nodes", np.float32).reshape(-1, 12), g("tri_indices", np.int32).reshape(-1),
                     g("normals", np.float32).reshape(-1, 4), g("normals_indices", np.int32).reshape(-1),
                     g("materials", np.float32).reshape(-1, 44), g("tri_to_material", np.int32).reshape(-1),
                     g("scene_min", np.float32).reshape(3), g("scene_max", np.float32).reshape(3))

    @staticmethod
    def from_mesh(mesh: "Mesh", bvh: "Bvh") -> "Scene":
        m = mesh.arrays()
        return Scene(m["vertices"], m["indices"], bvh.nodes, bvh.tri_indices, m["normals"],
                     m["normals_indices"], m["materials"], m["tri_to_material"], m["scene_min"], m["scene_max"])


class Mesh:
    """Owning wrapper of rtamd::Mesh (Mesh.h:69-101)."""

    def __init__(self):
        self._h = lib().rt_mesh_create()
        if not self._h:
            raise RtError(-4, "rt_mesh_create")

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.rt_mesh_destroy(self._h)
            self._h = None

    @classmethod
    def cornell(cls) -> "Mesh":
        m = cls(); _check(lib().rt_mesh_gen_cornell(m._h)); return m

    @classmethod
    def torus_knot(cls, nu=256, nv=137) -> "Mesh":
        m = cls(); _check(lib().rt_mesh_gen_torus_knot(m._h, nu, nv)); return m

    @classmethod
    def heightfield(cls, nx=500, nz=1000, amplitude=10.0, seed=0x5EED, extent=(-100.0, 100.0, -100.0, 100.0)) -> "Mesh":
        m = cls(); _check(lib().rt_mesh_gen_heightfield(m._h, nx, nz, amplitude, seed, *extent)); return m

    @classmethod
    def random(cls, ntris, extent=80.0, size=6.0, seed=1) -> "Mesh":
        m = cls(); _check(lib().rt_mesh_gen_random(m._h, ntris, extent, size, seed)); return m

    @classmethod
    def load_obj(cls, path: str) -> "Mesh":
        m = cls(); _check(lib().rt_mesh_load_obj(m._h, path.encode())); return m

    @classmethod
    def load_dae(cls, path: str) -> "Mesh":
        """ColladaLoader::load + Mesh::init(ColladaLoader&) (ColladaLoader.cpp:13-593, Mesh.cpp:10-78)."""
        m = cls(); _check(lib().rt_mesh_load_dae(m._h, path.encode())); return m

    def save_dae(self, path: str) -> None:
        """Writes the Collada subset load_dae (and the reference loader) reads."""
        _check(lib().rt_mesh_save_dae(self._h, path.encode()))

    @classmethod
    def from_arrays(cls, vertices, indices, normals=None, normals_indices=None, materials=None,
                    tri_to_material=None) -> "Mesh":
        m = cls()
        v = np.ascontiguousarray(vertices, np.float32).reshape(-1, 4)
        i = np.ascontiguousarray(indices, np.int32).reshape(-1)
        n = None if normals is None else np.ascontiguousarray(normals, np.float32).reshape(-1, 4)
        ni = None if normals_indices is None else np.ascontiguousarray(normals_indices, np.int32).reshape(-1)
        mt = None if materials is None else np.ascontiguousarray(materials, np.float32).reshape(-1, 44)
        tm = None if tri_to_material is None else np.ascontiguousarray(tri_to_material, np.int32).reshape(-1)
        _check(lib().rt_mesh_set(m._h, _ptr(v), v.shape[0], _ptr(i), i.size, _ptr(n), 0 if n is None else n.shape[0],
                                 _ptr(ni), _ptr(mt), 0 if mt is None else mt.shape[0], _ptr(tm)))
        return m

    def append_grid(self, src: "Mesh", gx: int, gz: int, dx: float, dz: float, scale: float = 1.0):
        _check(lib().rt_mesh_append_grid(self._h, src._h, gx, gz, dx, dz, scale))
        return self

    def arrays(self) -> dict:
        v = rt_mesh_view()
        _check(lib().rt_mesh_view_get(self._h, C.byref(v)))

        def cp(p, n, dt, w):
            if n == 0:
                return np.zeros((0, w) if w > 1 else 0, dt)
            buf = (C.c_char * (n * w * 4)).from_address(p)
            a = np.frombuffer(buf, dtype=dt).copy()
            return a.reshape(-1, w) if w > 1 else a
        return {
            "vertices": cp(v.vertices, v.num_vertices, np.float32, 4),
            "indices": cp(v.indices, v.num_indices, np.int32, 1),
            "normals": cp(v.normals, v.num_normals, np.float32, 4),
            "normals_indices": cp(v.normals_indices, v.num_indices, np.int32, 1),
            "materials": cp(v.materials, v.num_materials, np.float32, 44),
            "tri_to_material": cp(v.tri_to_material, v.num_indices // 3, np.int32, 1),
            "scene_min": np.array(list(v.scene_min), np.float32),
            "scene_max": np.array(list(v.scene_max), np.float32),
        }

    @property
    def num_triangles(self) -> int:
        v = rt_mesh_view()
        _check(lib().rt_mesh_view_get(self._h, C.byref(v)))
        return v.num_indices // 3

    def build_bvh(self, max_leaf: int = 8, threads: int = 0) -> "Bvh":
        h = C.c_void_p()
        _check(lib().rt_bvh_build(self._h, max_leaf, threads, C.byref(h)))
        return Bvh(h)

    def build_sbvh(self, threads: int = 0) -> "Bvh":
        """The reference's SplitBVHBuilder BVH (SplitBVHBuilder.cpp:41-476 + BVH_Cuda.h:87-137), same bytes."""
        h = C.c_void_p()
        _check(lib().rt_bvh_build_sbvh(self._h, threads, C.byref(h)))
        return Bvh(h)

    def load_bvh(self, path: str) -> "Bvh":
        h = C.c_void_p()
        _check(lib().rt_bvh_load(self._h, path.encode(), C.byref(h)))
        return Bvh(h)

    def camera_params(self, w: int, h: int, radius: float = 200.0, extra_alpha: float = 0.0,
                      extra_beta: float = 0.0, light_pos=None, light_color=None) -> rt_params:
        p = rt_params()
        lp = None if light_pos is None else np.asarray(light_pos, np.float32)
        lc = None if light_color is None else np.asarray(light_color, np.float32)
        _check(lib().rt_camera_params(self._h, w, h, radius, extra_alpha, extra_beta, _ptr(lp), _ptr(lc),
                                      C.byref(p)))
        return p


class Camera:
    """The reference's orbit camera (Camera.cpp:6-68) + updateCamera (RayTracer.cpp:609-672)."""

    def __init__(self, radius: float = 200.0):
        self._h = lib().rt_camera_create(radius)
        if not self._h:
            raise MemoryError("rt_camera_create")

    def add_rotate(self, da: float, db: float) -> None:
        _check(lib().rt_camera_add_rotate(self._h, da, db))

    def add_radius(self, dr: float) -> None:
        _check(lib().rt_camera_add_radius(self._h, dr))

    def params(self, mesh: "Mesh", w: int, h: int) -> rt_params:
        p = rt_params()
        _check(lib().rt_camera_frame_params(self._h, mesh._h, w, h, None, None, C.byref(p)))
        return p

    def __del__(self):
        if getattr(self, "_h", None):
            lib().rt_camera_destroy(self._h)
            self._h = None


class Bvh:
    def __init__(self, handle):
        self._h = handle
        v = rt_bvh_view()
        _check(lib().rt_bvh_view_get(self._h, C.byref(v)))
        nb = v.num_nodes * 48
        self.nodes = np.frombuffer((C.c_char * nb).from_address(v.nodes), np.float32).copy().reshape(-1, 12)
        nr = v.num_tri_indices
        self.tri_indices = (np.frombuffer((C.c_char * (nr * 4)).from_address(v.tri_indices), np.int32).copy()
                            if nr else np.zeros(0, np.int32))
        self.max_depth = v.max_depth
        self.num_leaves = v.num_leaves
        self.build_seconds = v.build_seconds

    def save(self, mesh: Mesh, path: str):
        _check(lib().rt_bvh_save(self._h, mesh._h, path.encode()))

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.rt_bvh_destroy(self._h)
            self._h = None


class Renderer:
    """One rt_ctx = one GPU (RayTraceData + command queue in the reference)."""

    def __init__(self, device: int = 0):
        h = C.c_void_p()
        _check(lib().rt_create(device, C.byref(h)))
        self._h = h
        self.device = device

    def close(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.rt_destroy(self._h)
            self._h = None

    __del__ = close

    def upload(self, s: Scene):
        self._scene_keepalive = s
        _check(lib().rt_upload_scene(
            self._h, _ptr(s.vertices), s.vertices.shape[0], _ptr(s.indices), s.indices.size,
            _ptr(s.nodes), s.nodes.shape[0], _ptr(s.tri_indices), s.tri_indices.size,
            _ptr(s.normals), s.normals.shape[0], _ptr(s.normals_indices), _ptr(s.materials), s.materials.shape[0],
            _ptr(s.tri_to_material)), self._h)

    def scene_image_size(self) -> int:
        """Bytes of this ctx's scene image (rt_scene_image_size)."""
        v = C.c_uint64()
        _check(lib().rt_scene_image_size(self._h, C.byref(v)), self._h)
        return v.value

    def pack_scene(self, d_image: int, nbytes: int, stream: Optional[int] = None) -> None:
        """Copy the uploaded scene's device layouts into the device buffer at d_image."""
        _check(lib().rt_scene_image_pack(self._h, C.c_void_p(d_image), nbytes, C.c_void_p(stream or None)), self._h)

    def load_scene(self, d_image: int, nbytes: int, stream: Optional[int] = None) -> None:
        """Replace this ctx's scene by a scene image (from pack_scene, e.g. broadcast by rank 0)."""
        self._scene_keepalive = None
        _check(lib().rt_scene_image_load(self._h, C.c_void_p(d_image), nbytes, C.c_void_p(stream or None)), self._h)

    def fetch_counts(self, w: int, h: int, depth: int = 1, flags: int = 0):
        """rt_fetch_counts: one frame's record fetches (every launch of the frame, counting
        instantiation): lane-fetches, quad requests and wave-distinct records (inner / tri),
        wave iterations and those mixing inner and triangle steps."""
        out = (C.c_uint64 * 8)()
        _check(lib().rt_fetch_counts(self._h, w, h, depth, flags, out), self._h)
        return {"inner": int(out[0]), "tri": int(out[1]), "quad_inner": int(out[2]), "quad_tri": int(out[3]),
                "distinct_inner": int(out[4]), "distinct_tri": int(out[5]), "wave_instructions": int(out[6]),
                "mixed_instructions": int(out[7])}

    def chase_peak(self, table_records: int = 16384, iters: int = 512, group: int = 4):
        """rt_chase_peak: (ms per launch, waves) of the dependent-iteration latency roof."""
        ms, waves = C.c_float(), C.c_uint64()
        _check(lib().rt_chase_peak(self._h, table_records, iters, group, C.byref(ms), C.byref(waves)), self._h)
        return ms.value, waves.value

    def chase_latency(self, blocks: int, table_records: int = 16384, iters: int = 512, group: int = 4):
        """rt_chase_latency: the chase chain on `blocks` blocks of 4 waves (blocks = CUs: one wave
        per SIMD) -> (ms per launch, waves)."""
        ms, waves = C.c_float(), C.c_uint64()
        _check(lib().rt_chase_latency(self._h, table_records, iters, group, blocks, C.byref(ms), C.byref(waves)),
               self._h)
        return ms.value, waves.value

    def wave_timeline(self, w: int, h: int, depth: int = 1, flags: int = 0, frames: int = 1, cap_words: int = 1 << 25):
        """rt_wave_timeline: `frames` frames in flight with per-wave stamps.  Returns {"frame_ns",
        "first_ns", "frames", "launches": [per launch {"frame", "bounce", and arrays t0, t_trace, t_shade,
        t1, t2 (10 ns ticks relative to the earliest wave start of all launches, -1 = not stamped),
        main, prologue (loop trips, both rays), main_c, pro_c, main_s, pro_s (closest-hit / shadow),
        xcc, hwid, tag}]}."""
        buf = np.zeros(cap_words, np.uint32)
        used = C.c_uint64()
        _check(lib().rt_wave_timeline(self._h, w, h, depth, flags, frames, _ptr(buf), cap_words, C.byref(used)),
               self._h)
        nl = int(buf[0])
        rw = int(buf[4]) or 16   # words per wave record (16 before the memory-wait words)
        recs, off = [], 128
        for k in range(nl):
            nw = int(buf[8 + k])
            recs.append((int(buf[40 + k]), int(buf[72 + k]), buf[off:off + nw * rw].reshape(nw, rw).copy()))
            off += nw * rw
        base = min(int(r[:, 0].min()) for _, _, r in recs) if recs else 0
        out = []
        for fr, bo, r in recs:
            a = r.astype(np.int64)
            for j in (0, 1, 2, 3, 4, 12, 13):   # 32-bit tick wrap: relative to the first start (0 = not stamped)
                a[:, j] = np.where(r[:, j] == 0, -1, (r[:, j].astype(np.int64) - base) & 0xFFFFFFFF)
            out.append({"frame": fr, "bounce": bo, "t0": a[:, 0], "t_trace": a[:, 1], "t_shade": a[:, 2],
                        "t1": a[:, 3], "t2": a[:, 4], "main": a[:, 5] + a[:, 7], "prologue": a[:, 6] + a[:, 8],
                        "main_c": a[:, 5], "pro_c": a[:, 6], "main_s": a[:, 7], "pro_s": a[:, 8],
                        "xcc": a[:, 9] & 0xF, "hwid": a[:, 10], "tag": a[:, 11], "t_enter": a[:, 12],
                        "t_pro_end": a[:, 13]})
            if rw >= 20:   # RTK_TL_SPLIT builds: main-loop memory wait (ticks) and long-wait trips
                out[-1].update({"wait_c": a[:, 16], "wait_s": a[:, 17], "longwait_c": a[:, 18],
                                "longwait_s": a[:, 19]})
        return {"frame_ns": int(buf[2]), "first_ns": int(buf[3]), "frames": int(buf[1]), "launches": out,
                "split": bool(buf[5])}

    def copy_scene_from(self, src: "Renderer") -> None:
        """rt_scene_copy: this ctx gets src's uploaded scene (device to device / peer to peer)."""
        self._scene_keepalive = None
        _check(lib().rt_scene_copy(self._h, src._h), self._h)

    def gather_peak(self, table_records: int = 16384, iters: int = 256):
        """rt_gather_peak: (ms per launch, records read) of the random-record gather ceiling."""
        ms, n = C.c_float(), C.c_uint64()
        _check(lib().rt_gather_peak(self._h, table_records, iters, C.byref(ms), C.byref(n)), self._h)
        return ms.value, n.value

    def set_params(self, p):
        if isinstance(p, np.ndarray):
            p = array_to_params(p)
        _check(lib().rt_set_params(self._h, C.byref(p)), self._h)

    def render(self, w: int, h: int, depth: int = 3, flags: int = 0, aux: bool = False):
        out = np.zeros(w * h, np.uint32)
        if aux:
            d = max(depth, 1)
            hits = np.zeros((w * h, d, 2), np.int32)
            t = np.zeros((w * h, d), np.float32)
            rgb = np.zeros((w * h, 3), np.float32)
            ax = rt_aux(_ptr(hits).value, _ptr(t).value, _ptr(rgb).value)
            _check(lib().rt_render(self._h, w, h, depth, flags, _ptr(out), C.byref(ax)), self._h)
            return {"out": out, "hits": hits[:, :depth], "t": t[:, :depth], "rgb": rgb}
        _check(lib().rt_render(self._h, w, h, depth, flags, _ptr(out), None), self._h)
        return out

    def render_host_ptr(self, w: int, h: int, depth: int, flags: int, host_ptr: int) -> None:
        """rt_render into caller-owned host memory at `host_ptr` (w*h uint32, pageable or pinned)."""
        if not host_ptr:
            raise ValueError("render_host_ptr: null output pointer")
        _check(lib().rt_render(self._h, w, h, depth, flags, C.c_void_p(host_ptr), None), self._h)

    def render_device(self, w, h, depth, flags, d_out_ptr: int, tiling: Optional[rt_tiling] = None,
                      stream: Optional[int] = None, aux_ptrs=None):
        """Enqueue a frame on `stream` (a hipStream_t handle, e.g. torch.cuda.Stream().cuda_stream);
        None = the ctx's own stream.  torch's default stream (handle 0) is refused: the C ABI reads
        NULL as the ctx stream, which does not order with the legacy null stream."""
        _stream_arg(stream)
        ax = None if aux_ptrs is None else C.byref(rt_aux(*aux_ptrs))
        _check(lib().rt_render_device(self._h, w, h, depth, flags, None if tiling is None else C.byref(tiling),
                                      C.c_void_p(d_out_ptr), ax, C.c_void_p(stream or None)), self._h)

    def render_device_batch(self, w, h, depth, flags, params, d_out_ptr: int, frame_stride: int,
                            tiling: Optional[rt_tiling] = None, stream: Optional[int] = None):
        """rt_render_device_batch: len(params) frames (rt_params, or the 32-float arrays of
        params_to_array) in ONE launch, frame i with params[i] into d_out_ptr + 4 * i * frame_stride."""
        _stream_arg(stream)
        arr = (rt_params * max(1, len(params)))()
        for i, p in enumerate(params):
            arr[i] = p if isinstance(p, rt_params) else array_to_params(p)
        _check(lib().rt_render_device_batch(self._h, w, h, depth, flags, None if tiling is None else C.byref(tiling),
                                            arr, len(params), C.c_void_p(d_out_ptr), frame_stride,
                                            C.c_void_p(stream or None)), self._h)

    def render_batch(self, w: int, h: int, depth: int, flags: int, params, out_ptr: Optional[int] = None):
        """rt_render_batch: len(params) frames in one launch, synchronous; returns a (k, h*w) uint32
        array, or fills the host memory at out_ptr (k * w*h uint32, pageable or pinned)."""
        arr = (rt_params * max(1, len(params)))()
        for i, p in enumerate(params):
            arr[i] = p if isinstance(p, rt_params) else array_to_params(p)
        out = None
        if out_ptr is None:
            out = np.zeros((max(1, len(params)), w * h), np.uint32)
            out_ptr = out.ctypes.data
        _check(lib().rt_render_batch(self._h, w, h, depth, flags, arr, len(params), C.c_void_p(out_ptr)), self._h)
        return out

    def batch_launcher(self, w, h, depth, flags, tiling: Optional[rt_tiling] = None):
        """A callable (params_array, n, d_out_ptr, frame_stride, stream) -> None that enqueues n frames
        like render_device_batch; params_array is a ctypes (rt_params * >= n) array the caller fills."""
        fn = lib().rt_render_device_batch
        hdl, tl = self._h, (None if tiling is None else C.byref(tiling))
        w, h, depth, flags = C.c_uint32(w), C.c_uint32(h), C.c_int32(depth), C.c_uint32(flags)

        def launch(arr, n: int, d_out_ptr: int, frame_stride: int, stream: int) -> None:
            _stream_arg(stream)
            rc = fn(hdl, w, h, depth, flags, tl, arr, n, d_out_ptr, frame_stride, stream)
            if rc:
                _check(rc, hdl)
        return launch

    def frame_launcher(self, w, h, depth, flags, tiling: Optional[rt_tiling] = None):
        """A callable (d_out_ptr, stream) -> None that enqueues one frame like render_device,
        with its constant ctypes arguments built once (a per-frame host loop's fast path)."""
        fn = lib().rt_render_device
        hdl, tl = self._h, (None if tiling is None else C.byref(tiling))
        w, h, depth, flags = C.c_uint32(w), C.c_uint32(h), C.c_int32(depth), C.c_uint32(flags)

        def launch(d_out_ptr: int, stream: int) -> None:
            _stream_arg(stream)
            rc = fn(hdl, w, h, depth, flags, tl, d_out_ptr, None, stream)
            if rc:
                _check(rc, hdl)
        return launch

    def last_kernel_ms(self) -> float:
        """All kernels of the last frame (ms, HIP events on the launch stream)."""
        t = C.c_float()
        _check(lib().rt_last_timing(self._h, C.byref(t), None), self._h)
        return t.value

    def last_timing(self):
        """(frame kernels ms, fused render kernel alone ms) of the last frame."""
        t, k = C.c_float(), C.c_float()
        _check(lib().rt_last_timing(self._h, C.byref(t), C.byref(k)), self._h)
        return t.value, k.value

    def timing_average(self, n: int):
        """(frame kernels ms, fused render kernel ms) averaged over the last n frames (n <= 64)."""
        t, k = C.c_float(), C.c_float()
        _check(lib().rt_timing_average(self._h, n, C.byref(t), C.byref(k)), self._h)
        return t.value, k.value

    def last_deferred(self) -> int:
        """Traversals of the last frame that restarted with the general code (stack deeper than LDS)."""
        v = C.c_uint32()
        _check(lib().rt_last_deferred(self._h, C.byref(v)), self._h)
        return v.value

    def last_enqueue_time(self):
        """rt_last_enqueue_time: host steady-clock ns at the start / end of the last frame's enqueue."""
        b, e = C.c_uint64(), C.c_uint64()
        _check(lib().rt_last_enqueue_time(self._h, C.byref(b), C.byref(e)), self._h)
        return b.value, e.value

    def overflow_count(self) -> int:
        v = C.c_uint64()
        _check(lib().rt_overflow_count(self._h, C.byref(v)), self._h)
        return v.value


def render_tiled(renderers, w: int, h: int, depth: int = 3, flags: int = 0, out=None):
    """rt_render_tiled: one frame over the renderers' GPUs (8-row bands dealt round-robin, every
    context writing its rows straight into one host frame), synchronous.  `out`: None (a new
    pageable array), a numpy uint32 array, or an int address of w*h uint32 of host memory
    (pinned memory is written by the devices directly).  Returns the frame (numpy) or None for
    an address."""
    n = len(renderers)
    arr = (C.c_void_p * max(n, 1))(*[r._h.value if isinstance(r._h, C.c_void_p) else r._h for r in renderers])
    if out is None:
        out = np.zeros(w * h, np.uint32)
    ptr = out if isinstance(out, int) else _ptr(out)
    rc = lib().rt_render_tiled(arr, n, w, h, depth, flags, ptr)
    if rc:
        _check(rc, renderers[0]._h if n else None)
    return None if isinstance(out, int) else out


def tiled_direct_ok(dev_addrs) -> bool:
    """rt_tiled_direct_ok: whether rt_render_tiled writes the caller's buffer directly, given the
    device address each context's device resolved for it (0 = unmapped on that device)."""
    a = (C.c_uint64 * max(1, len(dev_addrs)))(*dev_addrs)
    return bool(lib().rt_tiled_direct_ok(len(dev_addrs), a))


def tiling_pixels(w: int, h: int, rank: int, nranks: int, band_rows: int) -> int:
    t = rt_tiling(rank, nranks, band_rows, 0)
    return int(lib().rt_tiling_pixels(w, h, C.byref(t)))


def rank_bands(h: int, rank: int, nranks: int, band_rows: int):
    """[(first global row, rows)] of the bands `rank` owns, in its buffer order
    (band b belongs to rank b % nranks; same rule as rt_tiling in include/rt_abi.h)."""
    nbands = (h + band_rows - 1) // band_rows
    return [(b * band_rows, min(band_rows, h - b * band_rows)) for b in range(rank, nbands, nranks)]


class Comm:
    """One RCCL communicator for the native band exchange (rt_comm_*, include/rt_abi.h):
    rank 0 makes the 128-byte id (Comm.unique_id()), every rank passes it to Comm(...)."""

    ID_BYTES = 128

    @staticmethod
    def unique_id() -> bytes:
        buf = (C.c_uint8 * Comm.ID_BYTES)()
        rc = lib().rt_comm_unique_id(buf, Comm.ID_BYTES)
        if rc:
            raise RtError(rc, lib().rt_comm_last_error().decode())
        return bytes(buf)

    def __init__(self, device: int, nranks: int, rank: int, uid: bytes):
        buf = (C.c_uint8 * Comm.ID_BYTES).from_buffer_copy(uid)
        h = C.c_void_p()
        rc = lib().rt_comm_create(device, nranks, rank, buf, Comm.ID_BYTES, C.byref(h))
        if rc:
            raise RtError(rc, lib().rt_comm_last_error().decode())
        self._h, self.rank, self.nranks = h, rank, nranks
        self._fn = lib().rt_frame_gather

    def frame_gather(self, d_bands: int, slot_pixels: int, d_slots: int, d_frame: int, w: int, h: int,
                     band_rows: int, stream: int) -> None:
        """rt_frame_gather: every rank's bands to rank 0's slots, then rank 0 assembles the frame."""
        _stream_arg(stream)
        rc = self._fn(self._h, d_bands, slot_pixels, d_slots or None, d_frame or None, w, h, band_rows, stream)
        if rc:
            raise RtError(rc, lib().rt_comm_last_error().decode())

    def frame_exchanger(self, frame_pixels: int, w: int, h: int, band_rows: int):
        """Callables (slot_wait(slot, stream), exchange(slot, nframes, d_bands, d_slots, d_frames,
        stream)) for rt_frame_slot_wait / rt_frame_exchange with their constant arguments bound
        once."""
        L, hdl = lib(), self._h
        fx, fw = L.rt_frame_exchange, L.rt_frame_slot_wait
        a = (C.c_uint64(frame_pixels),)
        b = (C.c_uint32(w), C.c_uint32(h), C.c_int32(band_rows))

        def slot_wait(slot: int, stream: int) -> None:
            _stream_arg(stream)
            rc = fw(hdl, slot, stream)
            if rc:
                raise RtError(rc, L.rt_comm_last_error().decode())

        def exchange(slot: int, nframes: int, d_bands: int, d_slots: int, d_frames: int, stream: int) -> None:
            _stream_arg(stream)
            rc = fx(hdl, slot, nframes, d_bands, *a, d_slots or None, d_frames or None, *b, stream)
            if rc:
                raise RtError(rc, L.rt_comm_last_error().decode())
        return slot_wait, exchange

    def ready_wait(self, slot: int, stream: int) -> None:
        """rt_frame_ready_wait: `stream` waits for slot's frame (rank 0: assembled)."""
        _stream_arg(stream)
        rc = lib().rt_frame_ready_wait(self._h, slot, stream)
        if rc:
            raise RtError(rc, lib().rt_comm_last_error().decode())

    def close(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.rt_comm_destroy(self._h)
            self._h = None

    __del__ = close


class SharedFrames:
    """Device memory of rank 0 mapped into the other ranks' processes (rt_ipc_*,
    include/rt_abi.h): rank 0 exports a buffer it owns (a torch tensor's data_ptr) with
    SharedFrames.export(...) -> (handle, offset); another process maps it with
    SharedFrames.open(device, handle, offset) and writes through .ptr."""

    HANDLE_BYTES = 64

    @staticmethod
    def export(device: int, d_ptr: int):
        buf = (C.c_uint8 * SharedFrames.HANDLE_BYTES)()
        off = C.c_uint64()
        rc = lib().rt_ipc_export(device, d_ptr, buf, SharedFrames.HANDLE_BYTES, C.byref(off))
        if rc:
            raise RtError(rc, lib().rt_comm_last_error().decode())
        return bytes(buf), off.value

    def __init__(self, device: int, base: int, offset: int):
        self.device, self.base, self.ptr = device, base, base + offset

    @classmethod
    def open(cls, device: int, handle: bytes, offset: int) -> "SharedFrames":
        buf = (C.c_uint8 * cls.HANDLE_BYTES).from_buffer_copy(handle)
        p = C.c_void_p()
        rc = lib().rt_ipc_open(device, buf, cls.HANDLE_BYTES, C.byref(p))
        if rc:
            raise RtError(rc, lib().rt_comm_last_error().decode())
        return cls(device, p.value, offset)

    def close(self):
        if getattr(self, "base", None) and _lib is not None:
            _lib.rt_ipc_close(self.device, self.base)
            self.base = self.ptr = None

    __del__ = close


def bands_putter(w: int, h: int, tiling: Optional[rt_tiling] = None):
    """A callable (d_bands, d_frame, stream) -> None for rt_bands_put with its constant
    arguments built once: this rank's bands into their rows of a (local or mapped) frame."""
    fn = lib().rt_bands_put
    tl = None if tiling is None else C.byref(tiling)
    a = (C.c_uint32(w), C.c_uint32(h), tl)

    def put(d_bands: int, d_frame: int, stream: int) -> None:
        _stream_arg(stream)
        rc = fn(d_bands, d_frame, *a, stream)
        if rc:
            _check(rc)
    return put


class SharedAlloc:
    """rt_shared_alloc: zeroed uncached device memory on `device` for rank 0's shared frames
    and sync block (peers write it over xGMI while rank 0's kernels poll and read it).
    .ptr; close() frees it."""

    def __init__(self, device: int, nbytes: int):
        p = C.c_void_p()
        rc = lib().rt_shared_alloc(device, nbytes, C.byref(p))
        if rc:
            raise RtError(rc, lib().rt_comm_last_error().decode())
        self.device, self.ptr, self.nbytes = device, p.value, nbytes

    def close(self):
        if getattr(self, "ptr", None) and _lib is not None:
            _lib.rt_shared_free(self.device, self.ptr)
            self.ptr = None

    __del__ = close


def copy_device(d_dst: int, d_src: int, nbytes: int, stream: int) -> None:
    """rt_copy_device: device-to-device copy on `stream`."""
    _stream_arg(stream)
    rc = lib().rt_copy_device(d_dst, d_src, nbytes, stream)
    if rc:
        raise RtError(rc, lib().rt_comm_last_error().decode())


def peer_access(device: int, peer: int) -> bool:
    """rt_peer_access: can `device` map `peer`'s memory (hipDeviceCanAccessPeer)."""
    v = C.c_int32()
    rc = lib().rt_peer_access(device, peer, C.byref(v))
    if rc:
        raise RtError(rc, lib().rt_comm_last_error().decode())
    return bool(v.value)


def frame_sync_words(nsets: int, nranks: int) -> int:
    return int(lib().rt_frame_sync_words(nsets, nranks))


class FrameSync:
    """Per-frame completion of the IPC band puts (rt_bands_put_sync / rt_frame_present).
    d_sync: rank 0's sync block (mapped on the other ranks), d_local: this rank's nsets
    counters; both zeroed by the caller before first use.  put(set, use, d_bands, d_frame,
    stream) every rank; present(set, use, stream) rank 0 after its own put (release(set, use,
    stream) after its consumers, when present was told not to release)."""

    def __init__(self, w: int, h: int, tiling: Optional[rt_tiling], nranks: int, nsets: int, d_sync: int,
                 d_local: int, timeout_ms: int = 0):
        L = lib()
        self._put, self._present = L.rt_bands_put_sync, L.rt_frame_present
        self._tl = None if tiling is None else C.byref(tiling)
        self._wh = (C.c_uint32(w), C.c_uint32(h))
        self.nranks, self.nsets, self.timeout = nranks, nsets, timeout_ms
        self.d_sync, self.d_local = d_sync, d_local

    def put(self, set_: int, use: int, d_bands: int, d_frame: int, stream: int) -> None:
        _stream_arg(stream)
        rc = self._put(d_bands, d_frame, *self._wh, self._tl, self.d_sync, self.d_local, self.nsets, set_, use,
                       self.timeout, stream)
        if rc:
            _check(rc)

    def present(self, set_: int, use: int, stream: int, release: bool = True) -> None:
        _stream_arg(stream)
        rc = self._present(self.d_sync, self.nsets, set_, use, self.nranks, self.timeout, 1 if release else 0, stream)
        if rc:
            _check(rc)

    def release(self, set_: int, use: int, stream: int) -> None:
        """rt_frame_release: after the frame's consumers on `stream` (present(..., release=False))."""
        _stream_arg(stream)
        _check(lib().rt_frame_release(self.d_sync, self.nsets, set_, use, stream))

    def status(self):
        """(status, frames presented): 0 = ok, 1 = a put timed out, 2 = a present timed out."""
        st, n = C.c_uint32(), C.c_uint32()
        _check(lib().rt_frame_sync_status(self.d_sync, C.byref(st), C.byref(n)))
        return st.value, n.value


def frame_checksum(d_frame: int, pixels: int, d_sum: int, stream: int) -> None:
    """rt_frame_checksum: add the frame's position-dependent 64-bit sum into *d_sum."""
    _stream_arg(stream)
    _check(lib().rt_frame_checksum(d_frame, pixels, d_sum, stream))


def _stream_arg(stream):
    if stream is not None and int(stream) == 0:
        raise ValueError("stream 0 (the null stream) is not accepted: the C ABI reads NULL as the ctx stream; "
                         "run under a torch.cuda.Stream")


def assemble_bands_device(d_frame: int, d_slots: int, slot_pixels: int, w: int, h: int, nranks: int,
                          band_rows: int, stream: int) -> None:
    """rt_assemble_bands: rank 0's band re-interleave as one HIP launch on `stream`
    (device pointers; d_slots = nranks equal slots of slot_pixels pixels)."""
    _stream_arg(stream)
    _check(lib().rt_assemble_bands(C.c_void_p(d_frame), C.c_void_p(d_slots), slot_pixels, w, h, nranks, band_rows,
                                   C.c_void_p(stream or None)))


def bands_assembler(w: int, h: int, nranks: int, band_rows: int, slot_pixels: int, frame_pixels: int = 0):
    """A callable (d_frames, d_slots, stream[, nframes]) -> None for rt_assemble_bands_batch
    with its constant arguments built once (frame_pixels 0 = slot_pixels: one frame per slot)."""
    fn = lib().rt_assemble_bands_batch
    a = (C.c_uint64(slot_pixels), C.c_uint64(frame_pixels or slot_pixels))
    b = (C.c_uint32(w), C.c_uint32(h), C.c_int32(nranks), C.c_int32(band_rows))

    def assemble(d_frames: int, d_slots: int, stream: int, nframes: int = 1) -> None:
        _stream_arg(stream)
        rc = fn(d_frames, d_slots, *a, nframes, *b, stream)
        if rc:
            _check(rc)
    return assemble


def assemble_bands(frame, chunks, w: int, h: int, band_rows: int):
    """Host restatement of rt_assemble_bands (tests): re-interleave per-rank band
    buffers into the frame.  `frame` is (h*w,) and chunks[r] holds rank r's bands in
    order (it may be longer than the bands, e.g. a padded gather slot); numpy arrays
    or torch tensors (device copies stay on the device)."""
    nranks = len(chunks)
    for r, ch in enumerate(chunks):
        row = 0
        for y0, n in rank_bands(h, r, nranks, band_rows):
            dst, src = frame[y0 * w:(y0 + n) * w], ch[row * w:(row + n) * w]
            if isinstance(frame, np.ndarray):
                dst[:] = src
            else:
                dst.copy_(src, non_blocking=True)
            row += n
    return frame
