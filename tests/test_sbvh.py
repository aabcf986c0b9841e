"""The reference's spatial-split BVH (SplitBVHBuilder + BVH_Cuda::build_from_bvh2).

Product: rt_bvh_build_sbvh (csrc/host/sbvh_builder.cpp, parallel).  Oracle:
oracle/sbvh_oracle.c, a step-for-step restatement of SplitBVHBuilder.cpp:41-476.
The reference builder itself does not compile here (pugixml absent), so the
oracle is pinned by the survey's probe of the real builder on cubes2.obj
(14,933 nodes, 23,836 tri refs; and the traversal work the real tree
costs per primary ray at 1024x768: 18.74 / 1.60 / 5.98, max stack 14) and by the
recorded digest of its output (tests/golden/sbvh_digests.json, made by
tests/golden/make_sbvh_digests.py; a regression lock, not a pin).
Bar: product bytes == oracle bytes.
"""
import hashlib
import json
import os

import numpy as np
import pytest

import rtamd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CUBES2 = "/root/reference/x64/Release/data/models/cubes2.obj"
DIGESTS = os.path.join(ROOT, "tests", "golden", "sbvh_digests.json")


def _oracle(mesh):
    from oracle import oracle
    a = mesh.arrays()
    return oracle.sbvh(a["vertices"], a["indices"])


def _same(mesh, threads=4):
    on, orf = _oracle(mesh)
    b = mesh.build_sbvh(threads)
    pn = np.ascontiguousarray(b.nodes).view(np.uint32).reshape(-1, 12)
    assert pn.shape == on.shape, f"node count {pn.shape[0]} vs oracle {on.shape[0]}"
    diff = np.argwhere((pn != on.view(np.uint32)).any(1)).ravel()
    assert diff.size == 0, f"nodes differ from the oracle at {diff[:5].tolist()}"
    assert np.array_equal(b.tri_indices, orf), "tri_indices differ from the oracle"
    return on, orf


def digest(nodes, refs):
    h = hashlib.sha256()
    h.update(np.ascontiguousarray(nodes).view(np.uint8).tobytes())
    h.update(np.ascontiguousarray(refs, np.int32).view(np.uint8).tobytes())
    return h.hexdigest()


def _meshes():
    return {
        "cornell": lambda: rtamd.Mesh.cornell(),
        "knot": lambda: rtamd.Mesh.torus_knot(96, 40),
        "heightfield": lambda: rtamd.Mesh.heightfield(70, 60, 10.0, 11),
        "random_splits": lambda: rtamd.Mesh.random(6000, 100.0, 12.0, 3),   # long triangles -> spatial splits
        "random_small": lambda: rtamd.Mesh.random(200, 20.0, 2.0, 4),
    }


@pytest.mark.parametrize("name", sorted(_meshes()))
def test_product_matches_oracle(name):
    _same(_meshes()[name]())


def test_spatial_splits_are_exercised():
    m = _meshes()["random_splits"]()
    _, refs = _same(m, threads=8)
    assert refs.size > m.num_triangles, "expected duplicated references from spatial splits"


def test_thread_count_does_not_change_bytes():
    m = rtamd.Mesh.random(30000, 100.0, 6.0, 21)
    a = m.build_sbvh(1)
    b = m.build_sbvh(16)
    assert np.array_equal(a.nodes.view(np.uint32), b.nodes.view(np.uint32))
    assert np.array_equal(a.tri_indices, b.tri_indices)


def test_degenerate_and_tiny_meshes():
    # zero, one and two triangles; a line-degenerate and a point-degenerate triangle
    # (removed by buildNode's degenerate filter, SplitBVHBuilder.cpp:120-132)
    v = np.array([[0, 0, 0, 1], [1, 0, 0, 1], [0, 1, 0, 1], [2, 2, 2, 1], [5, 0, 0, 1], [7, 0, 0, 1],
                  [0, 0, 9, 1]], np.float32)
    for idx in ([], [0, 1, 2], [0, 1, 2, 3, 4, 6], [0, 1, 2, 4, 5, 4, 3, 3, 3, 0, 2, 6]):
        m = rtamd.Mesh.from_arrays(v, np.array(idx, np.int32))
        _same(m)


def test_signed_zero_and_axis_planes():
    # some triangles lie in the y = 0 plane with -0 / +0 coordinates: growth order decides +-0 in boxes
    rng = np.random.default_rng(5)
    n = 300
    v = rng.uniform(-10, 10, (3 * n, 4)).astype(np.float32)
    v[:, 3] = 1
    planar = np.arange(n) % 4 == 0
    for k, z in enumerate((-0.0, 0.0, -0.0)):
        v[3 * np.flatnonzero(planar) + k, 1] = z
    v[3 * np.flatnonzero(~planar)[::2], 1] = -0.0
    m = rtamd.Mesh.from_arrays(v, np.arange(3 * n, dtype=np.int32))
    _same(m)


@pytest.mark.skipif(not os.path.exists(CUBES2), reason="reference data not present")
def test_oracle_pinned_by_survey_probe_on_cubes2():
    m = rtamd.Mesh.load_obj(CUBES2)
    nodes, refs = _same(m, threads=8)
    assert nodes.shape[0] == 14933 and refs.size == 23836   # SURVEY.md section 6, probe of the real builder
    want = json.load(open(DIGESTS))["cubes2_obj"]
    assert digest(nodes, refs) == want


@pytest.mark.skipif(not os.path.exists(CUBES2), reason="reference data not present")
def test_traversal_work_pinned_by_survey_probe_on_cubes2():
    """The survey ran the REAL SplitBVHBuilder and the reference's traversal order on cubes2.obj
    at the reference's 1024x768 with its default camera (SURVEY.md 6 / BASELINE.md: 18.74 inner
    visits, 1.60 leaves, 5.98 triangle tests per primary ray, max stack depth 14).  The product
    SBVH traversed by the oracle must do the same work: a structural pin on the tree beyond its
    node and reference counts (a different split or child order changes these averages)."""
    from oracle import oracle
    m = rtamd.Mesh.load_obj(CUBES2)
    s = rtamd.Scene.from_mesh(m, m.build_sbvh(8))
    w, h = 1024, 768   # RayTracer.cpp:39-40
    r = oracle.render(s, rtamd.params_to_array(m.camera_params(w, h)), w, h, depth=1, aux=False)
    st = r["stats"]
    pr = st["primary"]
    assert pr["rays"] == w * h
    assert round(pr["inner"] / pr["rays"], 2) == 18.74
    assert round(pr["leaf"] / pr["rays"], 2) == 1.60
    assert round(pr["tris"] / pr["rays"], 2) == 5.98
    assert st["max_stack"] == 14


def test_recorded_digests_of_synthetic_scenes():
    want = json.load(open(DIGESTS))
    for name, make in _meshes().items():
        if name in want:
            b = make().build_sbvh(4)
            assert digest(b.nodes, b.tri_indices) == want[name], name


def test_sbvh_renders_through_the_oracle_like_any_bvh():
    """The SBVH output is a valid BVH_Node_ array: the oracle traverses it (parity of the GPU
    path on it is in test_render_gpu.py)."""
    from oracle import oracle
    m = rtamd.Mesh.torus_knot(64, 24)
    s = rtamd.Scene.from_mesh(m, m.build_sbvh())
    p = rtamd.params_to_array(m.camera_params(48, 32))
    r = oracle.render(s, p, 48, 32, depth=2)
    assert (r["hits"][..., 0] >= 0).any()
