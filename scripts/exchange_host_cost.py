"""Host cost of each call of the native frame exchange (diagnostic): one rank, a config's scene,
frames on F streams cycling 2F slots, per call perf_counter averages of
rt_frame_slot_wait / rt_render_device / rt_frame_exchange.

  python scripts/exchange_host_cost.py [--frames 600] [--inflight 4] [--config c3]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "real-time-opencl-raytracer_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=600)
    ap.add_argument("--inflight", type=int, default=4)
    ap.add_argument("--config", default="c3")
    args = ap.parse_args()
    os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")
    import torch
    import rtamd
    from rtamd import configs

    cfg = configs.CONFIGS[args.config]
    mesh, bvh, _ = configs.make_scene(cfg, 16, "sbvh", False)
    r = rtamd.Renderer(0)
    r.upload(rtamd.Scene.from_mesh(mesh, bvh))
    w, h = cfg["w"], cfg["h"]
    r.set_params(rtamd.params_to_array(mesh.camera_params(w, h)))
    cap = (w * h + 3) // 4 * 4
    comm = rtamd.Comm(0, 1, 0, rtamd.Comm.unique_id())
    F = args.inflight
    NB = 2 * F
    streams = [torch.cuda.Stream() for _ in range(F)]
    outs = [torch.zeros(cap, dtype=torch.int32, device="cuda") for _ in range(NB)]
    slots = [torch.zeros(cap, dtype=torch.int32, device="cuda") for _ in range(NB)]
    frames = [torch.zeros(h * w, dtype=torch.int32, device="cuda") for _ in range(NB)]
    launch = r.frame_launcher(w, h, cfg["depth"], cfg["flags"], rtamd.rt_tiling(0, 1, 8, 0))
    slot_wait, xchg = comm.frame_exchanger(cap, w, h, 8)
    sh = [s.cuda_stream for s in streams]
    tw = tl = tx = 0.0
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for n in range(args.frames):
        k, j = n % F, n % NB
        a = time.perf_counter()
        slot_wait(j, sh[k])
        b = time.perf_counter()
        launch(outs[j].data_ptr(), sh[k])
        c = time.perf_counter()
        xchg(j, outs[j].data_ptr(), slots[j].data_ptr(), frames[j].data_ptr(), sh[k])
        d = time.perf_counter()
        tw += b - a
        tl += c - b
        tx += d - c
    host = time.perf_counter() - t0
    torch.cuda.synchronize()
    total = time.perf_counter() - t0
    n = args.frames
    print(f"per frame: slot_wait {tw / n * 1e3:.4f} ms, render {tl / n * 1e3:.4f} ms, exchange {tx / n * 1e3:.4f} ms; "
          f"host {host / n * 1e3:.4f} ms, elapsed {total / n * 1e3:.4f} ms")
    comm.close()


if __name__ == "__main__":
    main()
