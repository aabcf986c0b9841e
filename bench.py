"""Benchmark of the render hot path (BASELINE.json metric).

One step = one frame: every rank renders its screen bands of the 1080p frame
(rt_render_device, inputs resident in HBM), then the packed pixel bands are
gathered to rank 0 over RCCL and re-interleaved into the frame.
`value` = rays traced by all ranks (primary + shadow) / max-over-ranks time.

    python bench.py [--gpus N --steps K --warmup W --config c3]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "real-time-opencl-raytracer_amd")
for _p in (PKG, ROOT):
    if _p not in sys.path:
        sys.path.insert(0, _p)

# Frames in flight run on separate streams; HIP maps streams onto GPU_MAX_HW_QUEUES hardware
# queues (4 by default, and exported as 4 on the GPU boxes; shared with torch's and the
# library's own streams), so with four frames in flight two would share a queue and
# serialise.  Raised to at least 8, before HIP starts (measured: 1/8 shard 0.075 -> 0.055 ms).
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < 8:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"

METRIC = "Mrays/sec (primary+1 shadow) @1080p, 1M-tri SAH BVH; 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)
# C3 terrain extent: fills the default camera's 1080p view (Camera.cpp:6-19)
HF_EXT = (-150.0, 650.0, -150.0, 650.0)

CONFIGS = {
    # BASELINE.json configs[2] -- the metric's configuration
    "c3": dict(scene="heightfield", nx=500, nz=1000, amp=10.0, seed=0x5EED, ext=HF_EXT, w=1920, h=1080, depth=1, flags=0,
               desc="C3: 1M-tri value-noise heightfield (500x1000 cells x2, seed 0x5EED), 1920x1080, "
                    "primary + 1 shadow ray"),
    # configs[1]: ~70k-tri mesh, primary only
    "c2": dict(scene="knot", nu=256, nv=137, w=1920, h=1080, depth=1, flags=1,
               desc="C2: 70,144-tri torus knot, 1920x1080, primary rays only"),
    # configs[3]: C3 scene at 4K (multi-GPU scaling curve)
    "c4": dict(scene="heightfield", nx=500, nz=1000, amp=10.0, seed=0x5EED, ext=HF_EXT, w=3840, h=2160, depth=1, flags=0,
               desc="C4: C3 scene at 3840x2160, primary + 1 shadow ray"),
    # configs[4]: 10M tris (10 x C3 on a 5x2 grid), depth 3 (primary + 2 bounces, shadows), in
    # the wavefront mode with per-bounce ray sorting, as the config names it: flags 8 | 32 =
    # RT_FLAG_WAVEFRONT | RT_FLAG_WF_SORT
    "c5": dict(scene="hf10", nx=500, nz=1000, amp=10.0, seed=0x5EED, ext=(-80.0, 80.0, -200.0, 200.0), w=1920, h=1080, depth=3,
               flags=8 | 32,
               dae=False,  # a 1 GB Collada text file is not worth the round trip; built in memory
               desc="C5: 10M-tri merged scene (10 x C3 on a 5x2 grid), 1920x1080, 3 bounces with shadows, "
                    "wavefront mode with per-bounce ray sorting"),
    # the same without the sort: faster here, the sort costs more than the coherence it buys;
    # with frames in flight the per-bounce launches also beat the fused kernel
    "c5u": dict(scene="hf10", nx=500, nz=1000, amp=10.0, seed=0x5EED, ext=(-80.0, 80.0, -200.0, 200.0), w=1920, h=1080, depth=3,
                flags=8, dae=False,
                desc="C5 scene and frame, wavefront mode without ray sorting"),
}


def make_scene(cfg, threads, builder="sbvh", via_dae=True):
    """The config's synthetic mesh; with via_dae (configs C2-C4) it is written
    as the reference-subset Collada file and read back through the ColladaLoader path
    (rt_mesh_save_dae / rt_mesh_load_dae), as the reference application loads its scene."""
    import tempfile
    import rtamd
    if cfg["scene"] == "heightfield":
        mesh = rtamd.Mesh.heightfield(cfg["nx"], cfg["nz"], cfg["amp"], cfg["seed"], cfg["ext"])
    elif cfg["scene"] == "knot":
        mesh = rtamd.Mesh.torus_knot(cfg["nu"], cfg["nv"])
    elif cfg["scene"] == "hf10":
        tile = rtamd.Mesh.heightfield(cfg["nx"], cfg["nz"], cfg["amp"], cfg["seed"], cfg["ext"])
        mesh = rtamd.Mesh()
        mesh.append_grid(tile, 5, 2, 160.0, 400.0, 1.0)
    else:
        raise ValueError(cfg["scene"])
    if via_dae and cfg.get("dae", True):
        with tempfile.TemporaryDirectory() as td:
            path = os.path.join(td, "scene.dae")
            mesh.save_dae(path)
            mesh = rtamd.Mesh.load_dae(path)
    t0 = time.time()
    bvh = mesh.build_sbvh(threads) if builder == "sbvh" else mesh.build_bvh(8, threads)
    return mesh, bvh, time.time() - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)   # 0.2 s of frames: steady state, not clock ramp-up
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--band-rows", type=int, default=8,
                    help="rows per screen band (bands dealt round-robin to ranks; 8 = one tile row)")
    ap.add_argument("--dist", action="store_true", help="use the process-group gather path even at N = 1")
    ap.add_argument("--gather", default="native", choices=["torch", "native"],
                    help="band exchange at N > 1: torch.distributed gather (async, RCCL) + rt_assemble_bands, or "
                         "the library's own RCCL communicators on the frame's stream (rt_frame_gather)")
    ap.add_argument("--inflight", type=int, default=4,
                    help="frames in flight (one stream each): frame i+1 renders while frame i drains / gathers")
    ap.add_argument("--shard", default="", help="R/N: render only rank R's bands of an N-way split (diagnostic)")
    ap.add_argument("--direct", action="store_true", help="skip the Collada write/read of the scene")
    ap.add_argument("--bvh", default="sbvh", choices=["sbvh", "binned"],
                    help="sbvh: the reference's SplitBVHBuilder (same bytes); binned: binned-SAH object splits")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="budget of the CPU baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--extra-flags", type=int, default=0, help="OR-ed into rt_render flags (A/B: 2 = HW math, "
                    "4 = IEEE-division slab test)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    import rtamd

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    if ndev and local >= ndev:   # rehearsal with more ranks than devices (not a bench setting)
        local %= ndev
    # --dist: the distributed frame path (process group, gather, assembly) even at N = 1,
    # to exercise it on a one-GPU box
    use_dist = world > 1 or args.dist
    if use_dist:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    cfg = CONFIGS[args.config]
    w, h, depth, flags = cfg["w"], cfg["h"], cfg["depth"], cfg["flags"] | args.extra_flags

    host_threads = max(1, min(16, (os.cpu_count() or 1)) // max(1, world))
    mesh, bvh, build_s = make_scene(cfg, host_threads, args.bvh, not args.direct)
    scene = rtamd.Scene.from_mesh(mesh, bvh)
    params = rtamd.params_to_array(mesh.camera_params(w, h))
    r = rtamd.Renderer(local)
    r.upload(scene)
    r.set_params(params)

    # --shard R/N (diagnostic, world 1 only): render just shard R of an N-way band split,
    # i.e. one rank's kernel work at N GPUs without the gather
    shard_r, shard_n = rank, world
    if args.shard:
        if world != 1:
            raise SystemExit("--shard is a single-process diagnostic")
        shard_r, shard_n = (int(v) for v in args.shard.split("/"))
    tiling = rtamd.rt_tiling(shard_r, shard_n, args.band_rows, 0)
    npx = rtamd.tiling_pixels(w, h, shard_r, shard_n, args.band_rows)
    cap = rtamd.tiling_pixels(w, h, 0, shard_n, args.band_rows)  # rank 0 owns the most bands
    cap = (cap + 3) // 4 * 4                                     # 16-B aligned gather slots
    # Frames in flight: frame i runs on stream i % F (each stream has its own frame scratch in
    # the library, rt_render_device), so frame i+1's render overlaps frame i's tail and, at N > 1,
    # frame i's RCCL gather.  Every launch of a frame -- render, the gather's ordering (RCCL waits
    # on torch's current stream) and rank 0's assembly -- is on that frame's stream.  (torch's
    # default stream is handle 0, which the C ABI would read as "the ctx's own stream".)
    F = max(1, args.inflight)
    streams = [torch.cuda.Stream(dev) for _ in range(F)]
    torch.cuda.set_stream(streams[0])
    outs = [torch.zeros(cap, dtype=torch.int32, device=dev) for _ in range(F)]
    # rank 0: per in-flight frame one contiguous (world, cap) gather target, re-interleaved into
    # that frame's framebuffer by one rt_assemble_bands launch
    gbufs = [torch.zeros(world, cap, dtype=torch.int32, device=dev) for _ in range(F)] \
        if (use_dist and rank == 0) else None
    glists = [list(g.unbind(0)) for g in gbufs] if gbufs is not None else [None] * F
    frames = [torch.zeros(h * w, dtype=torch.int32, device=dev) for _ in range(F)] \
        if (rank == 0 and use_dist) else None

    # rays traced per frame by this rank (counted once with the aux planes)
    d = max(depth, 1)
    hits = torch.zeros(npx * d * 2, dtype=torch.int32, device=dev)
    tt = torch.zeros(npx * d, dtype=torch.float32, device=dev)
    rgb = torch.zeros(npx * 3, dtype=torch.float32, device=dev)
    r.render_device(w, h, depth, flags, outs[0].data_ptr(), tiling=tiling, stream=streams[0].cuda_stream,
                    aux_ptrs=(hits.data_ptr(), tt.data_ptr(), rgb.data_ptr()))
    torch.cuda.synchronize(dev)
    hv = hits.view(npx, d, 2)
    rays_local = int((hv[..., 0] != -2).sum().item()) + int((hv[..., 1] != -2).sum().item())
    prim_local = int((hv[:, 0, 0] != -2).sum().item())
    del hits, tt, rgb

    # One step = one frame: render this rank's bands -> (N > 1) async RCCL gather of the bands
    # to rank 0 -> rank 0 re-interleaves them into the frame.  A slot's previous frame is
    # finished (gather waited on, assembled) before the slot's buffers are reused.
    pending = [None] * F
    nstep = [0]
    # the per-frame host path, with everything constant bound once: at N = 8 a frame is
    # ~0.055 ms of GPU time, so the host's enqueue per frame has to stay well under that
    launch = r.frame_launcher(w, h, depth, flags, tiling)
    sh = [st.cuda_stream for st in streams]
    out_ptr = [o.data_ptr() for o in outs]
    if use_dist:
        pg = dist.distributed_c10d._get_default_group()
        gopts = dist.GatherOptions()
        gopts.rootRank = 0
        gopts.asyncOp = True
        g_out = [[glists[k]] if rank == 0 else [] for k in range(F)]
        g_in = [[o] for o in outs]
        if rank == 0:
            assemble = rtamd.bands_assembler(w, h, world, args.band_rows, cap)
            frame_ptr = [f.data_ptr() for f in frames]
            gbuf_ptr = [g.data_ptr() for g in gbufs]

    native = use_dist and args.gather == "native"
    comms = []
    if native:
        # one communicator per in-flight stream; rank 0's ids travel through the process
        # group's store.  If any rank cannot create them, every rank falls back to the
        # torch.distributed gather (agreed through an all-reduce, so no rank is left waiting).
        store = dist.distributed_c10d._get_default_store()
        ok = 1.0
        try:
            for k in range(F):
                key = f"rtamd_comm_{k}"
                if rank == 0:   # an empty id tells every rank not to enter the collective init
                    try:
                        uid0 = rtamd.Comm.unique_id()
                    except rtamd.RtError:
                        uid0 = b""
                    store.set(key, uid0)
                uid = bytes(store.get(key))
                if len(uid) != rtamd.Comm.ID_BYTES:
                    raise rtamd.RtError(-2, "rank 0 has no RCCL id")
                comms.append(rtamd.Comm(local, world, rank, uid))
        except rtamd.RtError as e:
            print(f"rank {rank}: native band exchange unavailable ({e}); using torch.distributed", file=sys.stderr)
            ok = 0.0
        flag = torch.tensor([ok], device=dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        if flag.item() < 1.0:
            native = False
            for c in comms:
                c.close()
            comms = []
        slots_ptr = [g.data_ptr() for g in gbufs] if rank == 0 else [0] * F
        fr_ptr = [f.data_ptr() for f in frames] if rank == 0 else [0] * F

    def finish(k):
        work, pending[k] = pending[k], None
        work.wait()   # orders streams[k] (the current stream) after the gather
        if rank == 0:
            assemble(frame_ptr[k], gbuf_ptr[k], sh[k])

    def step():
        k = nstep[0] % F
        nstep[0] += 1
        torch.cuda.set_stream(streams[k])
        if pending[k] is not None:
            finish(k)
        launch(out_ptr[k], sh[k])
        if native:     # gather + assembly on the frame's own stream: no cross-stream waits
            comms[k].frame_gather(out_ptr[k], cap, slots_ptr[k], fr_ptr[k], w, h, args.band_rows, sh[k])
        elif use_dist:   # dist.gather(outs[k], glists[k], dst=0, async_op=True) without its argument checks
            pending[k] = pg.gather(g_out[k], g_in[k], gopts)

    def drain():
        for j in range(F):
            k = (nstep[0] + j) % F   # oldest first
            if pending[k] is not None:
                torch.cuda.set_stream(streams[k])
                finish(k)

    for _ in range(args.warmup):
        step()
    drain()
    torch.cuda.synchronize(dev)
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    host_s = time.perf_counter() - t0   # host time to enqueue the steps (launch-bound if ~ elapsed)
    drain()
    torch.cuda.synchronize(dev)
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    torch.cuda.set_stream(streams[0])

    # check (untimed): rank 0's assembled frames equal its own one-rank render of the frame
    frame_ok = None
    if use_dist and rank == 0:
        full = torch.zeros(h * w, dtype=torch.int32, device=dev)
        r.render_device(w, h, depth, flags, full.data_ptr(), stream=streams[0].cuda_stream)
        torch.cuda.synchronize(dev)
        frame_ok = all(bool(torch.equal(full, f)) for f in frames)

    # per-launch kernel times of the timed steps, from the HIP events the library
    # records on the launch stream around each frame's kernels (ring of 64 frames)
    frame_ms_avg, kernel_ms_avg = r.timing_average(min(args.steps, 64))

    # (untimed for `value`) the reference's own boundary: rt_render, synchronous, the frame
    # read back into host memory (raytrace_gpgpu: launch + clFinish + clEnqueueReadBuffer,
    # RayTracer.cpp:330-344); pageable numpy and pinned host buffers
    host_boundary = None
    if world == 1 and not args.shard:
        def host_rate(buf_ptr, n=20):
            r.render_host_ptr(w, h, depth, flags, buf_ptr)
            t1 = time.perf_counter()
            for _ in range(n):
                r.render_host_ptr(w, h, depth, flags, buf_ptr)
            return (time.perf_counter() - t1) / n * 1e3
        pageable = np.zeros(w * h, np.uint32)
        pinned = torch.zeros(w * h, dtype=torch.int32, pin_memory=True)
        ms_pg = host_rate(pageable.ctypes.data)
        ms_pin = host_rate(pinned.data_ptr())
        host_boundary = {"api": "rt_render (synchronous, frame copied to host memory)",
                         "ms_per_frame_pageable": round(ms_pg, 4), "ms_per_frame_pinned": round(ms_pin, 4),
                         "mrays_per_s_pinned": round(rays_local / (ms_pin * 1e-3) / 1e6, 1)}

    if use_dist:
        t = torch.tensor([elapsed, float(rays_local), float(prim_local)], dtype=torch.float64, device=dev)
        tmax = t[:1].clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        tsum = t[1:].clone()
        dist.all_reduce(tsum, op=dist.ReduceOp.SUM)
        elapsed = float(tmax.item())
        rays_total, prim_total = float(tsum[0].item()), float(tsum[1].item())
        km = torch.tensor([kernel_ms_avg], dtype=torch.float64, device=dev)
        dist.all_reduce(km, op=dist.ReduceOp.MAX)
        kernel_ms_avg = float(km.item())
    else:
        rays_total, prim_total = float(rays_local), float(prim_local)

    ms_per_step = elapsed / args.steps * 1e3
    value = rays_total * args.steps / elapsed / 1e6

    if rank != 0:
        if world > 1:
            dist.barrier()
            for c in comms:
                c.close()
            dist.destroy_process_group()
        return

    # CPU oracle sample: algorithmic bytes/ray (roofline) + CPU baseline
    from oracle import oracle
    cpu = None
    bpr = None
    budget = args.cpu_seconds if (world == 1 and not args.no_cpu_baseline) else min(args.cpu_seconds, 5.0)
    ncores = min(16, os.cpu_count() or 1)
    tprobe = time.perf_counter()
    probe = oracle.render(scene, params, w, h, depth=depth, flags=flags, pixels=(0, (w * h) // 4093, 4093),
                          nthreads=ncores, aux=False)
    tprobe = time.perf_counter() - tprobe
    per_px = tprobe / max(1, (w * h) // 4093)
    npix_sample = int(min(w * h, max(1000, budget / max(per_px, 1e-9))))
    stride = max(1, (w * h) // npix_sample)
    npix_sample = (w * h) // stride
    # the sample is repeated (whole frames when the frame is cheaper than the budget)
    # until about `budget` seconds of CPU work have been timed
    t0 = time.perf_counter()
    reps = 0
    while True:
        samp = oracle.render(scene, params, w, h, depth=depth, flags=flags, pixels=(0, npix_sample, stride),
                             nthreads=ncores, aux=False)
        reps += 1
        cpu_s = time.perf_counter() - t0
        if cpu_s >= 0.6 * budget or reps >= 1000:
            break
    st = samp["stats"]
    cpu_rays = sum(st[k]["rays"] for k in ("primary", "shadow", "secondary"))
    kinds = [k for k in ("primary", "shadow", "secondary") if st[k]["rays"]]
    tot_bytes = sum(80.0 * st[k]["inner"] + 16.0 * st[k]["leaf"] + 64.0 * st[k]["tris"] for k in kinds)
    bpr = tot_bytes / max(1, cpu_rays)
    if world == 1 and not args.no_cpu_baseline:
        cpu = {"value": cpu_rays * reps / cpu_s / 1e6, "unit": "Mrays/s", "cores": ncores, "kind": "port",
               "sample": f"oracle/rt_oracle.c on every {stride}th pixel of the same frame ({npix_sample} px, "
                         f"{cpu_rays} rays) x {reps} repetition(s), {cpu_s:.1f} s, {ncores} threads"}

    # measured device copy rate (the roofline also against a measured stream-copy
    # peak): 1 GiB -> 1 GiB device-to-device copies, read + write bytes over HIP-event time
    src = torch.empty(1 << 28, dtype=torch.float32, device=dev)
    dst = torch.empty_like(src)
    dst.copy_(src)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(10):
        dst.copy_(src)
    ev1.record()
    ev1.synchronize()
    stream_copy_gbs = 10 * 2 * src.numel() * 4 / (ev0.elapsed_time(ev1) * 1e-3) / 1e9
    del src, dst

    # algorithmic bytes per launch = rays this launch traces x bytes/ray + 4 B/pixel output
    launch_rays = rays_total / max(1, world)
    launch_px = (w * h) / world if world > 1 else npx
    launch_bytes = launch_rays * bpr + 4.0 * launch_px
    achieved = launch_bytes / (kernel_ms_avg * 1e-3) / 1e9
    # with F frames in flight the launches overlap, so a launch's duration includes the time it
    # shares the GPU with its neighbours: the per-launch rate above under-reads the kernel's
    # throughput by up to ~F x.  The aggregate rate is the same bytes over the wall time per frame.
    achieved_aggregate = launch_bytes / (ms_per_step * 1e-3) / 1e9
    traffic = None
    pmc_path = os.path.join(ROOT, "profiles", f"pmc_{args.config}.json")
    if os.path.exists(pmc_path):
        try:
            traffic = json.load(open(pmc_path)).get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    res = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "Mrays/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic",
        "config": {"workload": cfg["desc"], "config": args.config, "triangles": mesh.num_triangles,
                   "bvh_nodes": int(bvh.nodes.shape[0]), "width": w, "height": h, "depth": depth,
                   "shadow": not (flags & 1), "rays_per_frame": int(rays_total),
                   "primary_rays_per_frame": int(prim_total),
                   "primary_mrays_per_s": round(prim_total * args.steps / elapsed / 1e6, 1),
                   "mpixels_per_s": round(w * h * args.steps / elapsed / 1e6, 1),"parallelism": (f"screen bands x{world} (RCCL gather)" if not args.shard
                                   else f"shard {args.shard} of the band split (diagnostic, no gather)"),
                   "band_rows": args.band_rows, "frames_in_flight": F,
                   "band_exchange": (None if not use_dist else "rt_frame_gather (library RCCL communicators)" if native
                                     else "torch.distributed gather (RCCL) + rt_assemble_bands"),
                   "gpu_max_hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES", "4")),
                   "host_enqueue_ms_per_step": round(host_s / args.steps * 1e3, 4), "bvh": ("SplitBVHBuilder (reference SBVH, same bytes)"
                                                        if args.bvh == "sbvh" else "binned SAH"),
                   "bvh_refs": int(bvh.tri_indices.size), "bvh_build_s": round(build_s, 3),
                   "scene_source": "Collada (rt_mesh_load_dae)" if (cfg.get("dae", True) and not args.direct)
                   else "in-memory generator"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "achieved_aggregate": round(achieved_aggregate, 2),
                     "frac_aggregate": round(achieved_aggregate / HBM_PEAK_GBS, 4),
                     "stream_copy_gbs": round(stream_copy_gbs, 1),
                     "frac_of_stream_copy": round(achieved / stream_copy_gbs, 4),
                     "launches_overlap": F > 1,
                     "bytes_per_ray": round(bpr, 1), "kernel_ms": round(kernel_ms_avg, 4),
                     "frame_kernels_ms": round(frame_ms_avg, 4),
                     "kernel": ("rtk_strict::first_bounce_kernel<true, false>" if depth == 1 else "rtk_strict::first_bounce_kernel<true, true>" if (flags & 8)
                                else "rtk_strict::render_kernel<true>")},
        "cpu_baseline": cpu,
    }
    if frame_ok is not None:
        res["config"]["gathered_frame_equals_single_rank_render"] = frame_ok
    if host_boundary is not None:
        res["config"]["host_boundary"] = host_boundary
    print(json.dumps(res))
    if use_dist:
        dist.barrier()
        for c in comms:
            c.close()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
