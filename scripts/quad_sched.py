"""Drive scripts/quad_sched_sim.c on a bench config (analysis only, CPU).

    python scripts/quad_sched.py --config c3 --stride 37 --policies 0 1 4 8
Prints, per scheduling policy, fetch units (the share_fetch cost model) and loop
iterations for the primary and shadow loops, relative to policy 0 (the current kernel).
"""
import argparse
import ctypes as C
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "real-time-opencl-raytracer_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--stride", type=int, default=37)
    ap.add_argument("--keymode", type=int, default=0, help="0 reference node index, 1 ref-derived approximation")
    ap.add_argument("--policies", type=int, nargs="+", default=[0, 1, 4, 8])
    a = ap.parse_args()
    so = os.path.join(ROOT, "scripts", "libquadsim.so")
    subprocess.run(["gcc", "-O2", "-shared", "-fPIC", "-o", so, os.path.join(ROOT, "scripts", "quad_sched_sim.c"),
                    "-lm", "-lpthread"], check=True)
    import bench
    import rtamd
    cfg = bench.CONFIGS[a.config]
    mesh, bvh, _ = bench.make_scene(cfg, 8, "sbvh", False)
    sc = rtamd.Scene.from_mesh(mesh, bvh)
    w, h = cfg["w"], cfg["h"]
    par = np.ascontiguousarray(rtamd.params_to_array(mesh.camera_params(w, h)), np.float32)
    arr = {k: np.ascontiguousarray(getattr(sc, k)) for k in ("vertices", "indices", "nodes", "tri_indices", "normals",
                                                             "normals_indices", "materials", "tri_to_material")}
    L = C.CDLL(so)
    vp = C.c_void_p
    p = lambda x: x.ctypes.data_as(vp)
    pol = np.array(a.policies, np.int32)
    out = np.zeros(4 * len(pol))
    out2 = np.zeros(2 * len(pol))
    ns = np.zeros(2, np.int64)
    L.quad_sim.argtypes = [vp, vp, vp, vp, C.c_int32, vp, C.c_int32, vp, vp, vp, vp, C.c_uint32, C.c_uint32, C.c_int,
                           C.c_int, vp, C.c_int, vp, vp, vp, C.c_int]
    L.quad_sim(p(par), p(arr["vertices"]), p(arr["indices"]), p(arr["nodes"]), arr["nodes"].shape[0],
               p(arr["tri_indices"]), arr["tri_indices"].size, p(arr["normals"]), p(arr["normals_indices"]),
               p(arr["materials"]), p(arr["tri_to_material"]), w, h, int(not (cfg["flags"] & 1)), a.stride, p(pol),
               len(pol), p(out), p(out2), p(ns), a.keymode)
    nw = out2[1]
    print(f"{a.config}: {int(nw)} waves sampled, lane steps primary {ns[0]}, shadow {ns[1]}")
    b = out[:4]
    for i, q in enumerate(pol):
        u = out[4 * i: 4 * i + 4]
        print(f"policy {q:2d}: units prim {u[0]/nw:8.1f} ({u[0]/b[0]:.3f})  shadow {u[2]/nw:8.1f} ({u[2]/max(b[2],1):.3f})  "
              f"total ({(u[0]+u[2])/(b[0]+b[2]):.3f})  iters prim {u[1]/nw:7.1f} ({u[1]/b[1]:.3f})  "
              f"shadow {u[3]/nw:6.1f} ({u[3]/max(b[3],1):.3f})  max wave iters {out2[2*i]:.0f}")
    print(f"lanes per unit at policy 0: {(ns[0]+ns[1])/(b[0]+b[2]):.2f}")


if __name__ == "__main__":
    main()
