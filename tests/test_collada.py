"""Collada path: rt_mesh_load_dae (csrc/host/collada.cpp) against the restatement
oracle/dae_oracle.py (ColladaLoader.cpp:13-593 + Mesh.cpp:10-78), and the DAE
writer (synthetic-scene generator).  Bar: every mesh array bit-identical.

Pins: the reference's own scene x64/Release/data/collada/cubes2.DAE has 23,392
triangles, 13 geometries and 13 effects; the rendered frame of
that scene is pinned against the reference kernel in tests/golden/cubes2_dae.npz.
"""
import os

import numpy as np
import pytest

import rtamd

CUBES2_DAE = "/root/reference/x64/Release/data/collada/cubes2.DAE"
KEYS = ("vertices", "indices", "normals", "normals_indices", "materials", "tri_to_material", "scene_min", "scene_max")


def _bits(x):
    x = np.asarray(x)
    return x.view(np.uint32) if x.dtype == np.float32 else x


def _same_as_oracle(path):
    from oracle import dae_oracle
    o = dae_oracle.load_dae(path)
    a = rtamd.Mesh.load_dae(path).arrays()
    for k in KEYS:
        assert np.shape(a[k]) == np.shape(o[k]), f"{k}: shape {np.shape(a[k])} vs oracle {np.shape(o[k])}"
        assert np.array_equal(_bits(a[k]), _bits(o[k])), f"{k} differs from the oracle"
    return a


@pytest.mark.skipif(not os.path.exists(CUBES2_DAE), reason="reference data not present")
def test_reference_scene_cubes2_dae():
    a = _same_as_oracle(CUBES2_DAE)
    assert a["indices"].size // 3 == 23392
    assert a["materials"].shape[0] == 13
    counts = np.bincount(a["tri_to_material"], minlength=13)
    assert sorted(counts.tolist()) == sorted([32] + [2760] * 8 + [320] * 4)


def _write(tmp_path, body, name="s.dae"):
    p = tmp_path / name
    p.write_text(body)
    return str(p)


EFFECT = """<effect id="{n}-fx" name="{n}"><profile_COMMON><technique sid="standard"><{t}>
  <diffuse><color sid="diffuse">{d}</color></diffuse><shininess><float sid="shininess">2.5</float></shininess>
</{t}></technique></profile_COMMON></effect>"""


def _geometry(gid, material, pos, nrm, tris, extra_inputs=""):
    pos_s = " ".join(f"{v:.9g}" for v in np.ravel(pos))
    nrm_s = " ".join(f"{v:.9g}" for v in np.ravel(nrm))
    ps = "".join(f"<p>{' '.join(str(i) for i in t)}</p>" for t in tris)
    return f"""<geometry id="{gid}-lib" name="{gid}Mesh"><mesh>
<source id="{gid}-Position"><float_array id="{gid}-Position-array" count="{np.size(pos)}">{pos_s}</float_array></source>
<source id="{gid}-Normal0"><float_array id="{gid}-Normal0-array" count="{np.size(nrm)}">{nrm_s}</float_array></source>
<source id="{gid}-UV0"><float_array id="{gid}-UV0-array" count="2">0 0</float_array></source>
<vertices id="{gid}-Vertex"><input semantic="POSITION" source="#{gid}-Position"/></vertices>
<polygons material="{material}" count="{len(tris)}">{extra_inputs}
<input semantic="VERTEX" offset="0" source="#{gid}-Vertex"/>
<input semantic="NORMAL" offset="1" source="#{gid}-Normal0"/>
<input semantic="TEXCOORD" offset="2" set="0" source="#{gid}-UV0"/>
{ps}</polygons></mesh></geometry>"""


def _doc(effects, geometries, nodes):
    return f"""<?xml version="1.0" encoding="utf-8"?>
<!-- handwritten test scene -->
<COLLADA xmlns="http://www.collada.org/2005/11/COLLADASchema" version="1.4.0">
<library_effects>{''.join(effects)}</library_effects>
<library_geometries>{''.join(geometries)}</library_geometries>
<library_visual_scenes><visual_scene id="s">{''.join(nodes)}</visual_scene></library_visual_scenes>
</COLLADA>"""


def _tri_geo(rng, n=6):
    pos = rng.uniform(-20, 20, (n, 3)).astype(np.float32)
    nrm = rng.normal(size=(n, 3)).astype(np.float32)
    tris = [[0, 1, 0, 1, 2, 0, 2, 3, 0], [3, 4, 0, 4, 5, 0, 5, 0, 0], [1, 1, 0, 3, 3, 0, 5, 5, 0]]
    return pos, nrm, tris


def _nodes():
    return [
        # rotate sids in the reference's order; sid rotateZ rotates about Y (i % 3 quirk)
        "<node id='a'><translate sid='translate'>1.5 -2 3.25</translate>"
        "<rotate sid='rotateZ'>0 0 1 30.5</rotate><rotate sid='jointOrientX'>1 0 0 -90.000000</rotate>"
        "<rotate sid='rotateY'>0 1 0 12</rotate><instance_geometry url='#g0-lib'/></node>",
        "<node id='b'><matrix>1 0 0 5  0 0.5 0 -1  0 0 2 0.25  0 0 0 1</matrix><instance_geometry url='#g1-lib'/></node>",
        "<node id='c'><translate>0 0 0</translate><instance_geometry url='#nothing'/></node>",  # -> geometry 0
    ]


def test_transforms_and_quirks(tmp_path):
    rng = np.random.default_rng(3)
    e = [EFFECT.format(n="red", t="cook-torrance", d="1 0 0 1"), EFFECT.format(n="blue", t="phong", d="0 0 1 1")]
    g = []
    for k, mat in enumerate(["red", "blue", "missing-material"]):
        pos, nrm, tris = _tri_geo(rng)
        g.append(_geometry(f"g{k}", mat, pos, nrm, tris))
    a = _same_as_oracle(_write(tmp_path, _doc(e, g, _nodes())))
    assert a["tri_to_material"].tolist() == [0] * 3 + [1] * 3 + [0] * 3   # unknown material -> index 0
    assert a["materials"].view(np.int32)[:, 0].tolist() == [2, 1]         # COOK_TORRANCE, PHONG


def test_effect_without_technique_shifts_indices(tmp_path):
    """An effect with neither cook-torrance nor phong keeps its index but is not appended
    (ColladaLoader.cpp:119-131): later materials point one past their record.  The
    reference would read out of bounds; the product reports it."""
    from oracle import dae_oracle
    rng = np.random.default_rng(6)
    e = [EFFECT.format(n="red", t="cook-torrance", d="1 0 0 1"),
         "<effect id='x-fx' name='flat'><profile_COMMON><technique sid='s'><lambert/></technique>"
         "</profile_COMMON></effect>",
         EFFECT.format(n="blue", t="phong", d="0 0 1 1")]
    g = []
    for k, mat in enumerate(["red", "blue", "red"]):
        pos, nrm, tris = _tri_geo(rng)
        g.append(_geometry(f"g{k}", mat, pos, nrm, tris))
    path = _write(tmp_path, _doc(e, g, _nodes()))
    o = dae_oracle.load_dae(path)
    assert o["materials"].shape[0] == 2 and 2 in o["tri_to_material"].tolist()
    with pytest.raises(rtamd.RtError):
        rtamd.Mesh.load_dae(path)


def test_text_forms_cdata_entities_missing_p(tmp_path):
    rng = np.random.default_rng(4)
    pos, nrm, tris = _tri_geo(rng)
    geo = _geometry("g0", "m", pos, nrm, tris).replace(
        "<p>1 1 0 3 3 0 5 5 0</p>", "<p><![CDATA[1 1 0 3 3 0 5 5 0]]></p>")
    geo = geo.replace(f'count="{len(tris)}"', f'count="{len(tris) + 2}"')  # two <p> missing -> zero indices
    eff = EFFECT.format(n="m", t="cook-torrance", d="0.25 0.5 &#48;.75 1")
    node = "<node id='n'><translate sid='translate'>\n 10\t20 30 </translate><instance_geometry url='#g0-lib'/></node>"
    a = _same_as_oracle(_write(tmp_path, _doc([eff], [geo], [node])))
    assert a["indices"].size == 15 and np.all(a["indices"][9:] == 0)
    assert np.allclose(a["materials"][0, 12:15], [0.25, 0.5, 0.75])


def test_missing_texcoord_is_an_error(tmp_path):
    rng = np.random.default_rng(5)
    pos, nrm, tris = _tri_geo(rng)
    geo = _geometry("g0", "m", pos, nrm, tris).replace(
        '<input semantic="TEXCOORD" offset="2" set="0" source="#g0-UV0"/>', "")
    path = _write(tmp_path, _doc([EFFECT.format(n="m", t="phong", d="1 1 1 1")], [geo],
                                 ["<node id='n'><translate>0 0 0</translate><instance_geometry url='#g0-lib'/></node>"]))
    with pytest.raises(rtamd.RtError):
        rtamd.Mesh.load_dae(path)


@pytest.mark.parametrize("make", ["knot", "heightfield", "cornell"])
def test_generator_round_trip(tmp_path, make):
    """save_dae writes what the reference loader reads; reading it back gives the same
    triangles (same order; single-material meshes keep their arrays exactly)."""
    m = {"knot": lambda: rtamd.Mesh.torus_knot(40, 12), "heightfield": lambda: rtamd.Mesh.heightfield(30, 20, 10.0, 9),
         "cornell": lambda: rtamd.Mesh.cornell()}[make]()
    path = str(tmp_path / f"{make}.dae")
    m.save_dae(path)
    b = _same_as_oracle(path)
    a = m.arrays()
    tri_a = a["vertices"][a["indices"], :3].reshape(-1, 3, 3)
    tri_b = b["vertices"][b["indices"], :3].reshape(-1, 3, 3)
    mat_a = a["tri_to_material"]
    order = np.argsort(mat_a, kind="stable")   # the writer groups triangles by material
    assert np.array_equal(_bits(tri_a[order] + 0.0), _bits(tri_b + 0.0))  # +0.0: identity transform drops -0
    assert np.array_equal(a["materials"], b["materials"])
    assert np.array_equal(np.sort(mat_a), b["tri_to_material"])
    if len(np.unique(mat_a)) == 1:
        assert np.array_equal(a["indices"], b["indices"])
