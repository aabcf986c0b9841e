"""Host-side scene tools: layouts, BVH invariants, camera, loaders, cache (CPU)."""
import os
import re

import numpy as np
import pytest

import rtamd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_DATA = "/root/reference/x64/Release/data"


def test_struct_sizes():
    import ctypes as C
    assert C.sizeof(rtamd.rt_params) == 128           # RayTracer.cpp:115-161
    m = rtamd.Mesh.cornell().arrays()
    assert m["materials"].shape[1] * 4 == 176          # Mesh.h:20-67
    b = rtamd.Mesh.cornell().build_bvh()
    assert b.nodes.shape[1] * 4 == 48                  # BVH_Cuda.h:12-29


def _check_bvh(mesh, bvh, max_leaf=8):
    a = mesh.arrays()
    nodes = bvh.nodes
    ni = nodes.view(np.int32)
    nn = nodes.shape[0]
    ntri = a["indices"].size // 3
    seen = np.zeros(ntri, np.int32)
    order = []

    def visit(i, lo=None, hi=None):
        order.append(i)
        mn, mx = nodes[i, 0:3], nodes[i, 4:7]
        if lo is not None:
            assert np.all(mn >= lo) and np.all(mx <= hi), "child box outside parent"
        l, r, off, cnt = ni[i, 8:12]
        if l >= 0:
            assert r >= 0 and off == -1 and cnt == 0
            assert l == i + 1, "left child must follow its parent (pre-order, BVH_Cuda.h:98-137)"
            visit(l, mn, mx)
            visit(r, mn, mx)
        else:
            assert r == -1 and 1 <= cnt <= max_leaf
            for k in range(off, off + cnt):
                t3 = bvh.tri_indices[k]
                assert t3 % 3 == 0
                seen[t3 // 3] += 1
                v = a["vertices"][a["indices"][t3:t3 + 3], :3]
                assert np.all(v >= mn) and np.all(v <= mx), "triangle outside its leaf box"
    visit(0)
    assert order == list(range(nn)), "nodes must be in pre-order, root = 0"
    return seen


@pytest.mark.parametrize("make", [lambda: rtamd.Mesh.cornell(), lambda: rtamd.Mesh.torus_knot(64, 32),
                                  lambda: rtamd.Mesh.heightfield(60, 90, 10.0, 5),
                                  lambda: rtamd.Mesh.random(3000, 50.0, 5.0, 9)])
def test_bvh_invariants(make):
    m = make()
    b = m.build_bvh()
    seen = _check_bvh(m, b)
    assert np.all(seen == 1), "every non-degenerate triangle exactly once"
    assert b.tri_indices.size == m.num_triangles


def test_bvh_deterministic_across_threads():
    m = rtamd.Mesh.heightfield(300, 300, 10.0, 1)
    b1 = m.build_bvh(8, 1)
    b8 = m.build_bvh(8, 8)
    assert np.array_equal(b1.nodes.view(np.uint32), b8.nodes.view(np.uint32))
    assert np.array_equal(b1.tri_indices, b8.tri_indices)


def test_bvh_drops_degenerate_refs():
    # SplitBVHBuilder.cpp:120-132: references whose box has < 2 non-zero extents are removed
    v = np.array([[0, 0, 0, 1], [1, 0, 0, 1], [2, 0, 0, 1],      # a line along x (degenerate)
                  [0, 0, 0, 1], [1, 0, 0, 1], [0, 1, 0, 1]], np.float32)
    m = rtamd.Mesh.from_arrays(v, np.arange(6, dtype=np.int32))
    b = m.build_bvh()
    assert list(b.tri_indices) == [3]


def test_bvh_leaf_sizes_and_escape():
    m = rtamd.Mesh.random(2000, 40.0, 10.0, 2)
    b = m.build_bvh(max_leaf=64)
    seen = _check_bvh(m, b, max_leaf=64)
    assert np.all(seen == 1)


def test_bvh_cache_roundtrip(tmp_path):
    m = rtamd.Mesh.torus_knot(40, 20)
    b = m.build_bvh()
    p = str(tmp_path / "knot.bvh")
    b.save(m, p)
    b2 = m.load_bvh(p)
    assert np.array_equal(b.nodes.view(np.uint32), b2.nodes.view(np.uint32))
    assert np.array_equal(b.tri_indices, b2.tri_indices)
    other = rtamd.Mesh.torus_knot(40, 21)
    with pytest.raises(rtamd.RtError):
        other.load_bvh(p)  # mesh hash mismatch


def test_default_camera_matches_reference():
    # Camera.cpp:6-19: radius 200, alpha 225 deg, beta 45 deg -> eye (-100, 141.42, -100)
    m = rtamd.Mesh.cornell()
    p = rtamd.params_to_array(m.camera_params(1024, 768)).reshape(8, 4)
    assert np.allclose(p[3, :3], [-100.0, 141.42136, -100.0], atol=1e-3)
    assert np.all(p[:, 3] == 1.0)
    assert np.allclose(p[4, :3], [-23, 200, 3]) and np.allclose(p[5, :3], [1, 1, 1])  # RayTracer.cpp:57-63
    # image plane: a spans the full width, b the full height, at distance 1 along the view
    half = np.tan(np.float32(60 * 3.1415 * 0.5 / 180))
    assert np.isclose(np.linalg.norm(p[0, :3]), 2 * half * 1024 / 768, rtol=1e-5)
    assert np.isclose(np.linalg.norm(p[1, :3]), 2 * half, rtol=1e-5)
    a = m.arrays()
    assert np.allclose(p[6, :3], a["scene_min"]) and np.allclose(p[7, :3], a["scene_max"])


def test_generators_sizes():
    assert rtamd.Mesh.cornell().num_triangles == 12
    assert rtamd.Mesh.torus_knot(256, 137).num_triangles == 70144
    m = rtamd.Mesh.heightfield(50, 100, 10.0, 0x5EED)
    assert m.num_triangles == 10000
    a = m.arrays()
    assert np.allclose(np.linalg.norm(a["normals"][:, :3], axis=1), 1.0, atol=1e-5)
    big = rtamd.Mesh()
    big.append_grid(rtamd.Mesh.torus_knot(16, 8), 5, 2, 10.0, 10.0)
    assert big.num_triangles == 10 * 256


def test_mesh_from_arrays_validates():
    with pytest.raises(rtamd.RtError):
        rtamd.Mesh.from_arrays(np.zeros((3, 4), np.float32), np.array([0, 1, 5], np.int32))


@pytest.mark.skipif(not os.path.isdir(REF_DATA), reason="reference assets not present")
def test_obj_loader_reference_assets():
    m = rtamd.Mesh.load_obj(os.path.join(REF_DATA, "models", "cubes2.obj"))
    assert m.num_triangles == 23392
    a = m.arrays()
    assert a["normals"].shape[0] == 3257
    assert np.allclose(np.linalg.norm(a["normals"][:, :3], axis=1), 1.0, atol=1e-5)
    s = rtamd.Mesh.load_obj(os.path.join(REF_DATA, "sphere.obj"))
    assert s.num_triangles == 80


def test_header_sizes_static_asserts():
    h = open(os.path.join(ROOT, "include", "rt_abi.h")).read()
    assert "sizeof(rt_bvh_node) == 48" in h and "sizeof(rt_material) == 176" in h and "sizeof(rt_params) == 128" in h
