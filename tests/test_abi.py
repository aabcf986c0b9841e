"""The C-ABI library loads and exports every function include/*.h declares (CPU;
no compute calls)."""
import ctypes as C
import os
import re
import subprocess

import pytest

import rtamd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared(header):
    txt = open(os.path.join(ROOT, "include", header)).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[A-Za-z_][\w\s\*]*?\b(rt_\w+)\s*\(", txt, flags=re.M)
    return sorted(set(names))


def test_headers_declare_expected_symbols():
    assert set(_declared("rt_abi.h")) == set(rtamd.ABI_SYMBOLS)
    assert set(_declared("rt_host.h")) == set(rtamd.HOST_SYMBOLS)


def test_library_exports_every_declared_symbol():
    lib = rtamd.lib()
    for name in _declared("rt_abi.h") + _declared("rt_host.h"):
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", rtamd.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT (rt_\w+)", out))
    assert set(_declared("rt_abi.h")) <= exported
    assert set(_declared("rt_host.h")) <= exported


def test_abi_version_and_errors_without_gpu():
    lib = rtamd.lib()
    assert lib.rt_abi_version() == 3   # 2: default arithmetic S_ref, RT_FLAG_STRICT_MATH; 3: rt_fetch_counts, IPC puts
    assert lib.rt_set_params(None, None) == -1
    assert lib.rt_render(None, 1, 1, 1, 0, None, None) == -1
    # rt_assemble_bands validates before any device call: null buffers, zero sizes, bad
    # rank counts, and a slot too small for rank 0's bands are RT_ERR_INVALID_ARG
    assert lib.rt_assemble_bands(None, None, 0, 0, 0, 0, 0, None) == -1
    assert lib.rt_assemble_bands(16, 16, 100, 10, 10, 0, 8, None) == -1
    assert lib.rt_assemble_bands(16, 16, 10, 10, 10, 2, 8, None) == -1   # rank 0 owns 8 rows = 80 px > 10
    with pytest.raises(ValueError):   # the wrapper refuses torch's null stream
        rtamd.assemble_bands_device(16, 16, 100, 10, 10, 1, 8, 0)
    assert rtamd.tiling_pixels(100, 50, 0, 1, 16) == 5000
    # bands of 16 rows over 50 rows, 3 ranks: rank 0 owns bands 0 and 3 (16 + 2 rows)
    assert rtamd.tiling_pixels(100, 50, 0, 3, 16) == 18 * 100
    assert rtamd.tiling_pixels(100, 50, 1, 3, 16) == 16 * 100
    assert sum(rtamd.tiling_pixels(100, 50, r, 3, 16) for r in range(3)) == 5000
    assert rtamd.tiling_pixels(100, 50, 5, 3, 16) == -1


def test_product_has_no_oracle_dependency():
    """The product library must not link or reference the oracle."""
    out = subprocess.run(["nm", "-D", rtamd.LIB_PATH], capture_output=True, text=True).stdout
    assert "oracle_" not in out
    deps = subprocess.run(["ldd", rtamd.LIB_PATH], capture_output=True, text=True).stdout
    assert "oracle" not in deps
    uses = re.compile(r"(^\s*(from|import)\s+oracle)|(#\s*include\s*[<\"][^>\"]*oracle)|liboracle|oracle_render|"
                      r"ref_ocl", re.M)
    for root, _, files in os.walk(os.path.join(ROOT, "real-time-opencl-raytracer_amd")):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".h", ".inc", "Makefile")):
                assert not uses.search(open(os.path.join(root, f)).read()), f


def test_multi_gpu_and_diagnostic_entry_points_reject_bad_arguments_without_gpu():
    """rt_render_tiled / rt_scene_copy / rt_render_device_batch / rt_wave_timeline / rt_chase_latency validate their
    arguments before any device call (RT_ERR_INVALID_ARG = -1, message in rt_last_error)."""
    import numpy as np
    lib = rtamd.lib()
    out = np.zeros(64, np.uint32)
    po = out.ctypes.data_as(C.c_void_p)
    two = (C.c_void_p * 2)()                       # two NULL contexts
    assert lib.rt_render_tiled(None, 1, 8, 8, 1, 0, po) == -1
    assert lib.rt_render_tiled(two, 0, 8, 8, 1, 0, po) == -1     # n = 0
    assert lib.rt_render_tiled(two, 65, 8, 8, 1, 0, po) == -1    # n > 64
    assert lib.rt_render_tiled(two, 2, 8, 8, 1, 0, po) == -1     # NULL entries
    assert b"NULL" in lib.rt_last_error(None)
    fake = (C.c_void_p * 2)(0x1000, 0x1000)        # never dereferenced: refused as a duplicate first
    assert lib.rt_render_tiled(fake, 2, 8, 8, 1, 0, po) == -1
    assert b"twice" in lib.rt_last_error(None)
    assert lib.rt_render_tiled(two, 2, 8, 8, 1, 0, None) == -1   # no output
    assert lib.rt_render_tiled(two, 2, 0, 8, 1, 0, po) == -1     # zero width
    assert lib.rt_render_tiled(two, 2, 8, 8, 9, 0, po) == -1     # depth > RT_MAX_DEPTH
    assert lib.rt_scene_copy(None, None) == -1
    cams = (rtamd.rt_params * 2)()
    assert lib.rt_render_device_batch(None, 8, 8, 1, 0, None, cams, 2, po, 64, None) == -1   # no context
    assert lib.rt_render_device_batch(None, 8, 8, 1, 0, None, None, 2, po, 64, None) == -1   # no params
    assert lib.rt_render_batch(None, 8, 8, 1, 0, cams, 2, po) == -1                          # no context
    used = C.c_uint64()
    assert lib.rt_wave_timeline(None, 8, 8, 1, 0, 1, po, 256, C.byref(used)) == -1
    ms, waves = C.c_float(), C.c_uint64()
    assert lib.rt_chase_latency(None, 16, 4, 4, 1, C.byref(ms), C.byref(waves)) == -1
    assert lib.rt_last_enqueue_time(None, C.byref(waves), C.byref(waves)) == -1


def test_tiled_frame_direct_or_staged_per_device():
    """rt_render_tiled writes the caller's buffer directly only when EVERY context's device resolved
    a device address for it (hipHostGetDevicePointer on that device) and each is 16-B aligned (the
    row-copy kernel's stores); one device that cannot map it, or a misaligned mapping, sends the
    whole frame through the portable pinned staging frame."""
    ok = rtamd.tiled_direct_ok
    base = 0x7F0000000000
    assert ok([base])
    assert ok([base + 16 * k for k in range(8)])                 # 8 devices, each its own mapping
    assert not ok([base, base, 0, base])                          # device 2 cannot address it
    assert not ok([0] * 8)                                        # pageable memory
    assert not ok([base, base + 4])                               # a mapping not 16-B aligned
    assert not ok([])
    assert rtamd.lib().rt_tiled_direct_ok(2, None) == 0
