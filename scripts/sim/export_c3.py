"""Writes the C3 scene (as bench.py builds it) in the raw form the wave-level simulators in
this directory read: c3_nodes.bin (rt_bvh_node, 48 B each), c3_vertices.bin (float4),
c3_indices.bin / c3_tri_indices.bin (int32), c3_params.bin (the 128-B Params of the
default camera at 1920x1080), c3_scene_min.bin / c3_scene_max.bin (3 floats).
Analysis only.  Usage: python scripts/sim/export_c3.py OUT_DIR [CONFIG]; then
gcc -O2 -o sim scripts/sim/wave_sim.c -lm && (cd OUT_DIR && /path/to/sim)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "real-time-opencl-raytracer_amd"))

import numpy as np  # noqa: E402
import rtamd  # noqa: E402
from rtamd import configs  # noqa: E402


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else "."
    name = sys.argv[2] if len(sys.argv) > 2 else "c3"   # another config's scene under the same file names
    os.makedirs(out, exist_ok=True)
    cfg = configs.CONFIGS[name]
    mesh, bvh, _ = configs.make_scene(cfg)
    s = rtamd.Scene.from_mesh(mesh, bvh)
    w = lambda name, a: np.ascontiguousarray(a).tofile(os.path.join(out, f"c3_{name}.bin"))  # noqa: E731
    w("nodes", s.nodes.astype(np.float32))
    w("vertices", s.vertices.astype(np.float32))
    w("indices", s.indices.astype(np.int32))
    w("tri_indices", s.tri_indices.astype(np.int32))
    w("params", rtamd.params_to_array(mesh.camera_params(cfg["w"], cfg["h"])).astype(np.float32))
    w("scene_min", s.scene_min.astype(np.float32))
    w("scene_max", s.scene_max.astype(np.float32))


if __name__ == "__main__":
    main()
