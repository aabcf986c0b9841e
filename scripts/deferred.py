"""Diagnostic: pixels the fast kernel hands back to the general kernel, per config."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "real-time-opencl-raytracer_amd"), ROOT]


def main():
    import torch
    import bench
    import rtamd
    for name in sys.argv[1:] or ["c3"]:
        cfg = bench.CONFIGS[name]
        mesh, bvh, _ = bench.make_scene(cfg, 16)
        w, h = cfg["w"], cfg["h"]
        r = rtamd.Renderer(0)
        r.upload(rtamd.Scene.from_mesh(mesh, bvh))
        r.set_params(rtamd.params_to_array(mesh.camera_params(w, h)))
        out = torch.zeros(w * h, dtype=torch.int32, device="cuda")
        for flags in (cfg["flags"], cfg["flags"] | rtamd.RT_FLAG_STATIC_ORDER):
            r.render_device(w, h, cfg["depth"], flags, out.data_ptr())
            torch.cuda.synchronize()
            print(name, "flags", flags, "restarted traversals:", r.last_deferred(), "timing", r.last_timing())
        r.close()


if __name__ == "__main__":
    main()
