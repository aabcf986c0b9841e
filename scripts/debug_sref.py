"""Where S_ref and the reference kernel's default build disagree at full size: the
differing pixels, their values, and what the other arithmetic modes / the division-form
slab test give there.  Diagnostic (GPU box): python scripts/debug_sref.py c2 [c3 ...]"""
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "real-time-opencl-raytracer_amd"), ROOT]

import rtamd  # noqa: E402
from rtamd import configs  # noqa: E402
from oracle import ref_ocl, oracle  # noqa: E402


def main(names):
    ren = rtamd.Renderer(0)
    for name in names:
        cfg = configs.CONFIGS[name]
        mesh, bvh, _ = configs.make_scene(cfg, threads=16)
        scene = rtamd.Scene.from_mesh(mesh, bvh)
        w, h = cfg["w"], cfg["h"]
        p = rtamd.params_to_array(mesh.camera_params(w, h))
        with tempfile.TemporaryDirectory() as td:
            ref = ref_ocl.render_subprocess(scene, p, w, h, "default", td)
        ren.upload(scene)
        ren.set_params(p)
        modes = {"ref": 0, "ref_div": 4, "hw": 2, "strict": 64}
        outs = {k: ren.render(w, h, depth=3, flags=v, aux=True) for k, v in modes.items()}
        bad = np.nonzero(outs["ref"]["out"] != ref)[0]
        print(f"== {name}: {len(bad)} pixels differ from the reference (S_ref)")
        for k in modes:
            print(f"   {k:8s}: {int(np.sum(outs[k]['out'] != ref))} differ")
        orc = oracle.render(scene, p, w, h, depth=3, pixels=(int(bad[0]), 1, 1)) if len(bad) else None
        for i in bad[:8]:
            x, y = i % w, i // w
            print(f" px {i} (x={x}, y={y}): reference {ref[i]:06x}")
            for k in modes:
                o = outs[k]
                print(f"   {k:8s} {o['out'][i]:06x} hits {o['hits'][i].tolist()} t {o['t'][i].tolist()} "
                      f"rgb {o['rgb'][i].tolist()}")
        if orc is not None:
            print("   oracle(first bad px)", hex(int(orc["out"][0])), orc["hits"][0].tolist(), orc["t"][0].tolist())


if __name__ == "__main__":
    main(sys.argv[1:] or ["c2"])
