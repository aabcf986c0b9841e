"""CPU restatement of the reference's Collada path (test infrastructure only).

ColladaLoader::load (ColladaLoader.cpp:13-593) + Mesh::init(ColladaLoader&)
(Mesh.cpp:10-78), written independently of the product loader
(real-time-opencl-raytracer_amd/csrc/host/collada.cpp) on Python's
xml.etree DOM.  Only tests/ import it, as the checker of rt_mesh_load_dae.

The reference links pugixml, which is not in the image (README:4), so the
reference loader cannot run here: this restatement is pinned by the counts the
survey recorded for the reference's own scene (x64/Release/data/collada/
cubes2.DAE: 23,392 triangles, 13 geometries, 13 effects)
and by the per-material triangle counts of that file, not by dumped arrays
("parity pinned by counts only").

Float text is read with the C library's strtof (what std::stof calls), float32
arithmetic is numpy float32 in the reference's evaluation order, and the
rotation sine / cosine are float(sin(double)), the same convention the product
uses (MSVC's sinf is unavailable: see collada.cpp).
"""
from __future__ import annotations

import ctypes
import math
import xml.etree.ElementTree as ET

import numpy as np

_libc = ctypes.CDLL(None)
_libc.strtof.restype = ctypes.c_float
_libc.strtof.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_char_p)]

F = np.float32
ATTRS = [("emission", "color", 4), ("ambient", "color", 4), ("diffuse", "color", 4), ("specular", "color", 4),
         ("shininess", "float", 1), ("reflective", "color", 4), ("reflectivity", "float", 1),
         ("transparent", "color", 4), ("transparency", "float", 1), ("glossiness", "float", 1)]


def _local(tag: str) -> str:
    return tag.split("}", 1)[1] if tag.startswith("{") else tag


def _child(node, name):
    if node is None:
        return None
    for c in node:
        if _local(c.tag) == name:
            return c
    return None


def _children(node, name):
    return [] if node is None else [c for c in node if _local(c.tag) == name]


def _text(node) -> str:
    return "" if node is None or node.text is None or node.text.strip() == "" else node.text


def _stof_array(s: str, n: int):
    """stof_array (ColladaLoader.h:20-31); None when nothing is written."""
    if len(s) < 1 or n < 1:
        return None
    buf = ctypes.create_string_buffer(s.encode())
    p = ctypes.cast(buf, ctypes.c_char_p)
    base = ctypes.addressof(buf)
    off = 0
    out = []
    end = ctypes.c_char_p()
    for _ in range(n):
        v = _libc.strtof(ctypes.c_char_p(base + off), ctypes.byref(end))
        e = ctypes.cast(end, ctypes.c_void_p).value - base
        if e == off:
            raise ValueError("stof: no conversion")
        out.append(F(v))
        off = e
    del p
    return out


class _Mat:
    """Matrix4x4 (Matrix4x4.cpp), row-major float32."""

    def __init__(self):
        self.m = [F(1) if i % 5 == 0 else F(0) for i in range(16)]

    def mul(self, b):
        r = [F(0)] * 16
        for i in range(4):
            for j in range(4):
                s = F(0)
                for k in range(4):
                    s = F(s + F(self.m[i * 4 + k] * b[k * 4 + j]))
                r[i * 4 + j] = s
        self.m = r

    def rotate(self, axis, a):
        s, c = F(math.sin(float(a))), F(math.cos(float(a)))
        z, o = F(0), F(1)
        if axis == 0:
            self.mul([o, z, z, z, z, c, s, z, z, -s, c, z, z, z, z, o])
        elif axis == 1:
            self.mul([c, z, -s, z, z, o, z, z, s, z, c, z, z, z, z, o])
        else:
            self.mul([c, s, z, z, -s, c, z, z, z, z, o, z, z, z, z, o])

    def apply(self, v):
        out = []
        for i in range(4):
            s = F(0)
            for j in range(4):
                s = F(s + F(v[j] * self.m[j * 4 + i]))
            out.append(s)
        return out


def load_dae(path: str) -> dict:
    root = ET.parse(path).getroot()
    if _local(root.tag) != "COLLADA":
        raise ValueError("no COLLADA root")
    effect_index, geometry_index = {}, {}
    materials = []
    for count, e in enumerate(_children(_child(root, "library_effects"), "effect")):      # :103-185
        effect_index[e.get("name", "")] = count
        tech = _child(_child(e, "profile_COMMON"), "technique")
        cur, technique = _child(tech, "cook-torrance"), 2
        if cur is None:
            cur, technique = _child(tech, "phong"), 1
        if cur is None:
            continue
        rec = np.zeros(44, np.float32)
        rec[0:4] = np.array([technique, 0, 0, 0], np.int32).view(np.float32)
        for i, (name, sub, n) in enumerate(ATTRS):
            vals = _stof_array(_text(_child(_child(cur, name), sub)), n)
            if vals is not None:
                rec[4 + 4 * i:4 + 4 * i + n] = vals
        materials.append(rec)

    geometries = []
    for count, g in enumerate(_children(_child(root, "library_geometries"), "geometry")):  # :200-290
        polys = _child(_child(g, "mesh"), "polygons")
        geometry_index[g.get("id", "")] = count
        npoly = int(polys.get("count"))
        effect = effect_index.setdefault(polys.get("material", ""), 0)
        ps = _children(polys, "p")
        tris = []
        for i in range(npoly):
            v9 = [0] * 9
            if i < len(ps) and _text(ps[i]):
                toks = _text(ps[i]).split()
                v9 = [int(t) for t in toks[:9]]
                if len(v9) != 9:
                    raise ValueError("<p> with fewer than 9 ints")
            tris.append((v9, effect))
        inputs = _children(polys, "input")[:3]

        def src(sem):
            for inp in inputs:
                if inp.get("semantic", "") == sem:
                    return inp.get("source", "")
            raise ValueError("missing input " + sem)
        mesh = _child(g, "mesh")

        def float_array(sid):
            for s in _children(mesh, "source"):
                if s.get("id", "") == sid:
                    return _child(s, "float_array")
            return None
        pos_id = ""
        for vtx in _children(mesh, "vertices"):
            if vtx.get("id", "") == src("VERTEX")[1:]:
                pos_id = (_child(vtx, "input").get("source", "") or "#")[1:]
                break

        def arr(fa):
            n = int(fa.get("count", "0")) if fa is not None else 0
            return _stof_array(_text(fa), n) or []
        geometries.append((tris, arr(float_array(pos_id)), arr(float_array(src("NORMAL")[1:]))))

    scene = []
    vs = _child(_child(root, "library_visual_scenes"), "visual_scene")
    for nd in _children(vs, "node"):                                                   # :428-545
        url = _child(nd, "instance_geometry").get("url", "")[1:]
        gi = geometry_index.setdefault(url, 0)
        M = _Mat()
        mx = _child(nd, "matrix")
        if mx is not None:
            m = _stof_array(_text(mx), 16)
            M.m = [m[j * 4 + i] for i in range(4) for j in range(4)]   # transponse
        else:
            rot = {r.get("sid", ""): r for r in _children(nd, "rotate")}
            for i, sid in enumerate(["jointOrientX", "jointOrientY", "jointOrientZ", "rotateX", "rotateZ", "rotateY"]):
                if sid not in rot:
                    continue
                angle = _stof_array(_text(rot[sid])[6:], 1)[0]
                rad = F(float(angle) * math.pi / 180.0)
                M.rotate(i % 3, rad)
            tr = _stof_array(_text(_child(nd, "translate")), 3) or [F(0)] * 3
            M.mul([F(1), F(0), F(0), F(0), F(0), F(1), F(0), F(0), F(0), F(0), F(1), F(0), tr[0], tr[1], tr[2], F(1)])
        scene.append((gi, M))

    g2s = {}
    for i in range(len(geometries)):                                                   # :583-592
        g2s[scene[i][0]] = i
    idx, nidx, t2m, verts, norms = [], [], [], [], []
    smin = smax = None
    for g, (tris, pos, nrm) in enumerate(geometries):                                  # Mesh.cpp:10-78
        vc, nc = len(verts), len(norms)
        for v9, eff in tris:
            idx += [vc + v9[0], vc + v9[3], vc + v9[6]]
            nidx += [nc + v9[1], nc + v9[4], nc + v9[7]]
            t2m.append(eff)
        M = scene[g2s.get(g, 0)][1]
        for j in range(0, len(pos) - 2, 3):
            r = M.apply([pos[j], pos[j + 1], pos[j + 2], F(1)])
            if smin is None:
                smin, smax = r[:3], r[:3]
            else:
                smin = [a if a < b else b for a, b in zip(smin, r[:3])]
                smax = [a if a > b else b for a, b in zip(smax, r[:3])]
            verts.append([r[0], r[1], r[2], F(1)])
        for j in range(0, len(nrm) - 2, 3):
            r = M.apply([nrm[j], nrm[j + 1], nrm[j + 2], F(0)])
            norms.append([r[0], r[1], r[2], F(1)])
    return dict(vertices=np.array(verts, np.float32).reshape(-1, 4), indices=np.array(idx, np.int32),
                normals=np.array(norms, np.float32).reshape(-1, 4), normals_indices=np.array(nidx, np.int32),
                materials=np.array(materials, np.float32).reshape(-1, 44), tri_to_material=np.array(t2m, np.int32),
                scene_min=np.array(smin, np.float32), scene_max=np.array(smax, np.float32))
