"""Benchmark of the render hot path (BASELINE.json metric).

One step = one frame: every rank renders its screen bands of the 1080p frame
(rt_render_device, inputs resident in HBM), then the packed pixel bands are
gathered to rank 0 over RCCL and re-interleaved into the frame.
`value` = rays traced by all ranks (primary + shadow) / max-over-ranks time.

    python bench.py [--gpus N --steps K --warmup W --config c3 --orbit 0.01]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

`--gpus N` without a torch.distributed environment starts torch.distributed.run with N
ranks as a child process (before anything touches the GPU) and passes rank 0's JSON
line through; under torchrun, WORLD_SIZE must equal --gpus.
"""
from __future__ import annotations

import argparse
import datetime
import glob
import json
import os
import socket
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "real-time-opencl-raytracer_amd")
for _p in (PKG, ROOT):
    if _p not in sys.path:
        sys.path.insert(0, _p)

METRIC = "Mrays/sec (primary+1 shadow) @1080p, 1M-tri SAH BVH; 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)
MATH = {0: "S_ref: the reference kernel as RayTracer.cpp builds it (bit-exact vs its gfx950 build)",
        64: "S_strict: the CPU oracle's arithmetic (RT_FLAG_STRICT_MATH)",
        2: "S_hw: the reference built with IEEE / and sqrt (RT_FLAG_HW_MATH)"}


def parse_args(argv=None):
    from rtamd.configs import CONFIGS
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)   # 0.2 s of frames: steady state, not clock ramp-up
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--orbit", type=float, default=0.0,
                    help="moving camera: add_rotate(ORBIT, 0) radians per frame, as the reference's mouse "
                         "drag does (RayTracer.cpp:553-565); 0 = the static default camera")
    ap.add_argument("--jitter", type=int, default=32,
                    help="static camera: cycle through this many sub-pixel jittered copies of it (frame n: camera "
                         "n %% J, the image plane shifted by a Halton(2,3) offset inside one pixel; camera 0 is the "
                         "unjittered one), so no two frames of a launch or of the frames in flight trace the same "
                         "rays; 1 = every frame the identical default camera")
    ap.add_argument("--band-rows", type=int, default=8,
                    help="rows per screen band (bands dealt round-robin to ranks; 8 = one tile row)")
    ap.add_argument("--dist", action="store_true", help="use the process-group gather path even at N = 1")
    ap.add_argument("--gather", default="ipc", choices=["ipc", "torch", "native"],
                    help="band exchange at N > 1.  ipc (default): no collective, every rank copies its bands "
                         "straight into rank 0's frame, mapped through a HIP IPC handle (rt_bands_put); falls back "
                         "to torch if any rank cannot map it.  torch: torch.distributed gather (async, RCCL) + "
                         "rt_assemble_bands.  native: the library's own RCCL communicator (rt_frame_exchange)")
    ap.add_argument("--pg", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend for setup and timing; gloo lets a rehearsal run N ranks on one "
                         "GPU (RCCL refuses two ranks on one device)")
    ap.add_argument("--gather-batch", type=int, default=4,
                    help="frames per exchange at N > 1: one gather carries B consecutive frames of a stream, so "
                         "the exchange's host cost is paid once per B frames")
    ap.add_argument("--local-batch", action="store_true",
                    help="diagnostic: batches of --gather-batch frames per stream at N = 1 too (no exchange)")
    ap.add_argument("--frames-per-launch", type=int, default=0,
                    help="render each batch of K frames (K <= 8) with ONE launch (rt_render_device_batch: the "
                         "longest tiles of all K frames first; depth 1, or the wavefront mode); the frames in flight are then "
                         "--inflight launches of K frames each.  0 (default): 4 at depth 1, 8 in the wavefront mode, else 1")
    ap.add_argument("--hang-timeout", type=float, default=600.0,
                    help="N > 1: a rank that has not finished this many seconds after joining the process group "
                         "exits with status 3 (a stuck collective ends the run instead of hanging it)")
    ap.add_argument("--inflight", type=int, default=4,
                    help="frames in flight (one stream each): frame i+1 renders while frame i drains / gathers")
    ap.add_argument("--shard", default="", help="R/N: render only rank R's bands of an N-way split (diagnostic)")
    ap.add_argument("--direct", action="store_true", help="skip the Collada write/read of the scene")
    ap.add_argument("--bvh", default="sbvh", choices=["sbvh", "binned"],
                    help="sbvh: the reference's SplitBVHBuilder (same bytes); binned: binned-SAH object splits")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="budget of the CPU baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true",
                    help="skip the fetch trace and the gather ceiling (profiling passes: keeps other kernels out)")
    ap.add_argument("--extra-flags", type=int, default=0,
                    help="OR-ed into rt_render flags (A/B: 64 = S_strict math, 2 = S_hw math, 4 = division-form "
                         "slab test, 16 = static block order)")
    ap.add_argument("--warmup-seconds", type=float, default=0.3,
                    help="after the --warmup frames, keep warming up until this much wall time of frames has run "
                         "(clock ramp-up after the idle scene setup)")
    ap.add_argument("--max-extra-warmup", type=int, default=4096, help="cap on the time-based extra warm-up frames")
    ap.add_argument("--frame-check", default="final", choices=["final", "every"],
                    help="N > 1 / --dist: final = every frame rank 0 holds at the end is compared with its own "
                         "one-rank render of that frame's camera; every = also a checksum of every presented frame, "
                         "taken when rank 0 saw it complete (ipc exchange)")
    ap.add_argument("--sync-timeout-ms", type=int, default=10000,
                    help="ipc exchange: bound on a put's wait for its frame set and on rank 0's wait for a frame")
    ap.add_argument("--inject-fault", default="none",
                    choices=["none", "wrong-bands", "drop-put", "drop-put-warmup", "no-peer", "open-fails",
                             "slow-setup"],
                    help="test only (ipc exchange, N > 1): the last rank puts frame 4's bands from another frame's "
                         "buffer (wrong-bands: the frame check must fail), or skips its put of frame 4 (drop-put: "
                         "frame delivery must fail by timeout), or of frame 1, a warm-up frame (drop-put-warmup: "
                         "the warm-up check must move every rank to the torch.distributed gather); or, at set-up, "
                         "its peer-access check says no (no-peer) or it maps rank 0's frames from a corrupted "
                         "handle, so rt_ipc_open fails (open-fails): every rank must take the torch.distributed "
                         "gather; or it finishes its set-up --slow-setup-s seconds late (slow-setup: past the "
                         "exchange bound; the ranks start the warm-up together, so the run must complete on the "
                         "IPC exchange)")
    ap.add_argument("--slow-setup-s", type=float, default=3.0, help="the slow-setup fault's delay")
    ap.add_argument("--no-setup-barrier", action="store_true",
                    help="test only: leave out the barrier before the warm-up (the round-4 flow), so a late rank's "
                         "set-up eats into rank 0's bounded wait for the first frame")
    ap.add_argument("--hw-queues", type=int, default=16,
                    help="raise GPU_MAX_HW_QUEUES to at least this before HIP starts (frames in flight need a "
                         "hardware queue each, beside torch's and RCCL's streams); 0 = keep the inherited value")
    ap.add_argument("--probe-launch", action="store_true",
                    help="launcher check without a GPU: every rank joins a gloo group and rank 0 reports the world")
    return ap.parse_args(argv)


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launcher_cmd(n: int, argv, port: int):
    """torch.distributed.run with n ranks of this script on one node (the driver's form)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)


def _probe(args):
    """--probe-launch: the rendezvous of the launched ranks, with gloo on the CPU."""
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    ranks = [None] * world
    dist.all_gather_object(ranks, {"rank": rank, "local_rank": int(os.environ.get("LOCAL_RANK", "0"))})
    t = torch.ones(1)
    dist.all_reduce(t)
    if rank == 0:
        print(json.dumps({"probe": True, "n_gpus": world, "gpus_arg": args.gpus, "all_reduce": float(t.item()),
                          "ranks": ranks}))
    dist.destroy_process_group()


def host_cpu_share():
    """The host cores this process may use: its CPU affinity, capped by the cgroup's CPU quota
    (a GPU box gives each GPU's job a share of a many-core host: os.cpu_count() reports the
    whole machine, the quota what the job can actually run on).  OMP_NUM_THREADS is used only
    when neither is readable."""
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = os.cpu_count() or 1
    quota = None
    try:   # cgroup v2: "max 100000" or "<quota> <period>"
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = float(q) / float(per)
    except (OSError, ValueError):
        try:   # cgroup v1
            q = float(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = float(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    omp = int(os.environ.get("OMP_NUM_THREADS") or 0) or None
    if quota is not None:
        cores, source = max(1, min(affinity, int(quota + 0.5))), "cgroup CPU quota"
    elif omp is not None and omp < affinity:
        cores, source = omp, "OMP_NUM_THREADS (no cgroup quota readable)"
    else:
        cores, source = affinity, "CPU affinity"
    return {"cores": cores, "source": source, "affinity": affinity, "cgroup_quota": quota,
            "omp_num_threads": omp, "os_cpu_count": os.cpu_count()}


def halton(i, b):
    f, x = 1.0, 0.0
    while i > 0:
        f /= b
        x += f * (i % b)
        i //= b
    return x


def jittered_cameras(p, w, h, n):
    """n copies of the camera Params p (32 floats), copy k with its image plane shifted by a
    sub-pixel offset (Halton(2,3) point k, centred: k = 0 is p itself): image_pos = c + a xf + b yf
    with xf = (x - 0.5) / w (volumeRender.cl:1169-1190), so c + a dx / w + b dy / h moves every
    primary ray by (dx, dy) pixels, |dx|, |dy| < 0.5."""
    import numpy as np
    out = np.repeat(p.reshape(1, 32), n, axis=0).astype(np.float32)
    q = p.reshape(8, 4).astype(np.float64)
    for k in range(1, n):
        dx, dy = halton(k, 2) - 0.5, halton(k, 3) - 0.5
        out[k, 8:11] = (q[2, :3] + q[0, :3] * (dx / w) + q[1, :3] * (dy / h)).astype(np.float32)
    return out


_SYNC = []   # the run's rtamd.FrameSync (ipc exchange), for the failure report


def _sync_state():
    if not _SYNC:
        return "none (no IPC exchange set up)"
    try:
        st, presented = _SYNC[0].status()
        return f"status {st} (0 ok, 1 a put timed out, 2 a present timed out), {presented} frames presented"
    except Exception as e:   # the device may be the thing that failed
        return f"unreadable ({e})"


def _hang_exit(rank, seconds):
    print(f"bench.py: rank {rank} still running {seconds:.0f} s after joining the process group; exiting; "
          f"frame-sync block: {_sync_state()}", file=sys.stderr, flush=True)
    os._exit(3)


def main():
    args = parse_args()
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        # N ranks requested from a plain `python bench.py --gpus N`: one process per GPU via
        # torch.distributed.run, started before this process touches the GPU
        rc = subprocess.call(launcher_cmd(args.gpus, sys.argv[1:], _free_port()),
                             env=dict(os.environ, MASTER_ADDR="127.0.0.1"))
        sys.exit(rc)
    world = int(world_env or "1")
    if world != args.gpus:
        sys.exit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}: the ranks must be the GPUs asked for")
    if args.probe_launch:
        _probe(args)
        return
    # the result is the ONE line on stdout: everything else the process writes to fd 1 (RCCL's
    # version banner on the first communicator, library messages) goes to stderr
    result_out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)
    try:
        run(args, world, result_out)
    except BaseException as e:
        # every failed rank says so on its own stderr, with the frame-sync block as it stands (the
        # round-4 3-rank abort left only the launcher's summary: DESIGN.md 8); then the failure goes on
        if not (isinstance(e, SystemExit) and e.code in (0, None)):
            print(f"bench.py: rank {os.environ.get('RANK', '0')} failed: {type(e).__name__}: {e}; "
                  f"frame-sync block: {_sync_state()}", file=sys.stderr, flush=True)
        raise


def run(args, world, result_out=None):
    # Frames in flight run on separate streams; HIP maps streams onto GPU_MAX_HW_QUEUES hardware
    # queues (4 by default, and exported as 4 on the GPU boxes), shared with torch's, RCCL's
    # and the library's own streams: two frame streams on one queue serialise.  Raised to at
    # least 16 before HIP starts (measured: 4 -> 8 took a 1/8 shard from 0.075 to 0.055 ms;
    # with an RCCL process group's streams also in the pool, 8 -> 16 took rank 0's 1/8-shard
    # frame from 0.071 to 0.045 ms).  Under rocprofv3 the profiler's preload starts HIP first,
    # so the profiling scripts set it in their own environment; the JSON says which applied.
    # --hw-queues 0 keeps the inherited value; the JSON reports both.
    q_in = os.environ.get("GPU_MAX_HW_QUEUES")
    inherited = int(q_in) if q_in else 4
    hw_queues = {"inherited": q_in or "unset (HIP default 4)", "effective": inherited, "set_by_bench": False}
    if args.hw_queues and inherited < args.hw_queues:
        os.environ["GPU_MAX_HW_QUEUES"] = str(args.hw_queues)
        hw_queues.update(effective=args.hw_queues, set_by_bench=True)

    import numpy as np
    import torch
    import torch.distributed as dist
    import rtamd
    from rtamd import configs

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    if ndev and local >= ndev:   # rehearsal with more ranks than devices (not a bench setting)
        local %= ndev
    # --dist: the distributed frame path (process group, gather, assembly) even at N = 1,
    # to exercise it on a one-GPU box
    use_dist = world > 1 or args.dist
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if use_dist:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        dist.init_process_group(args.pg, device_id=dev if args.pg == "nccl" else None,
                                timeout=datetime.timedelta(seconds=args.hang_timeout))
        watchdog = threading.Timer(args.hang_timeout, _hang_exit, (rank, args.hang_timeout))
        watchdog.daemon = True
        watchdog.start()
    pg_cpu = args.pg == "gloo"

    def bcast(t):   # device tensors through the process group (gloo: staged through host memory)
        if pg_cpu:
            c = t.cpu()
            dist.broadcast(c, src=0)
            t.copy_(c)
        else:
            dist.broadcast(t, src=0)

    def allreduce(t, op):
        if pg_cpu:
            c = t.cpu()
            dist.all_reduce(c, op=op)
            t.copy_(c)
        else:
            dist.all_reduce(t, op=op)

    cfg = configs.CONFIGS[args.config]
    w, h, depth, flags = cfg["w"], cfg["h"], cfg["depth"], cfg["flags"] | args.extra_flags
    math_flags = flags & (64 | 2)
    cpu_share = host_cpu_share()
    host_threads = cpu_share["cores"]
    nframes = args.warmup + args.steps

    # ---- scene: rank 0 builds it (Collada round trip + the reference's SBVH) and uploads it;
    # at N > 1 its device image is broadcast over RCCL and every other rank loads it ----
    r = rtamd.Renderer(local)
    mesh = bvh = None
    build_s = 0.0
    t_scene = time.perf_counter()
    if rank == 0:
        mesh, bvh, build_s = configs.make_scene(cfg, host_threads, args.bvh, not args.direct)
        r.upload(rtamd.Scene.from_mesh(mesh, bvh))
        if args.orbit:
            cam = rtamd.Camera()
            plist = []
            for f in range(nframes):
                if f > 0:
                    cam.add_rotate(args.orbit, 0.0)
                plist.append(rtamd.params_to_array(cam.params(mesh, w, h)))
            ptab = np.stack(plist)
        else:
            ptab = jittered_cameras(rtamd.params_to_array(mesh.camera_params(w, h)), w, h, max(1, args.jitter))
    scene_bytes = 0
    if world > 1:
        nb = torch.zeros(2, dtype=torch.int64, device=dev)
        if rank == 0:
            nb[0] = r.scene_image_size()
            nb[1] = ptab.shape[0]
        bcast(nb)
        scene_bytes = int(nb[0].item())
        img = torch.empty(scene_bytes, dtype=torch.uint8, device=dev)
        pt = torch.empty((int(nb[1].item()), 32), dtype=torch.float32, device=dev)
        if rank == 0:
            r.pack_scene(img.data_ptr(), scene_bytes, torch.cuda.current_stream().cuda_stream)
            pt.copy_(torch.from_numpy(ptab))
        bcast(img)
        bcast(pt)
        if rank != 0:
            torch.cuda.synchronize(dev)
            r.load_scene(img.data_ptr(), scene_bytes)
            ptab = pt.cpu().numpy()
        del img, pt
    scene_s = time.perf_counter() - t_scene
    r.set_params(ptab[0])

    # --shard R/N (diagnostic, world 1 only): render just shard R of an N-way band split,
    # i.e. one rank's kernel work at N GPUs without the gather; with --dist
    # (R = 0) also rank 0's exchange work at N GPUs: its own slot gathered, the whole frame
    # assembled from N slots (the other N-1 slots hold no peer data: no frame check)
    shard_r, shard_n = rank, world
    if args.shard:
        if world != 1:
            raise SystemExit("--shard is a single-process diagnostic")
        shard_r, shard_n = (int(v) for v in args.shard.split("/"))
        if use_dist and shard_r != 0:
            raise SystemExit("--dist --shard R/N: only R = 0 (rank 0's exchange work)")
    tiling = rtamd.rt_tiling(shard_r, shard_n, args.band_rows, 0)
    npx = rtamd.tiling_pixels(w, h, shard_r, shard_n, args.band_rows)
    cap = rtamd.tiling_pixels(w, h, 0, shard_n, args.band_rows)  # rank 0 owns the most bands
    cap = (cap + 3) // 4 * 4                                     # 16-B aligned gather slots
    # Frames in flight: batch i of B frames runs on stream i % F (each stream has its own frame
    # scratch in the library, rt_render_device), so its renders overlap the other streams' frames
    # and, at N > 1, the RCCL gathers of earlier batches.  (torch's default stream is handle 0,
    # which the C ABI would read as "the ctx's own stream".)
    F = max(1, args.inflight)
    native = use_dist and args.gather == "native"
    comms = []
    if native:
        # ONE communicator per rank (rt_frame_exchange: gathers in frame order on its own
        # stream); rank 0's id travels through the process group's store.  If any rank cannot
        # create it, every rank falls back to the torch.distributed gather (agreed through an
        # all-reduce, so no rank is left waiting).
        store = dist.distributed_c10d._get_default_store()
        ok = 1.0
        try:
            if rank == 0:   # an empty id tells every rank not to enter the collective init
                try:
                    uid0 = rtamd.Comm.unique_id()
                except rtamd.RtError:
                    uid0 = b""
                store.set("rtamd_comm", uid0)
            uid = bytes(store.get("rtamd_comm"))
            if len(uid) != rtamd.Comm.ID_BYTES:
                raise rtamd.RtError(-2, "rank 0 has no RCCL id")
            comms.append(rtamd.Comm(local, world, rank, uid))
        except rtamd.RtError as e:
            print(f"rank {rank}: native band exchange unavailable ({e}); using torch.distributed", file=sys.stderr)
            ok = 0.0
        flag = torch.tensor([ok], device=dev)
        allreduce(flag, dist.ReduceOp.MIN)
        if flag.item() < 1.0:
            native = False
            for c in comms:
                c.close()
            comms = []
    ipc = use_dist and args.gather == "ipc"
    tgather = use_dist and not native and not ipc
    # frames per exchange: a batch of B consecutive frames renders on one stream into one
    # (B, cap) buffer and one gather carries the whole batch, so the exchange's host cost
    # (~0.05 ms per gather with its event waits; a 1/8 shard's frame is ~0.05 ms) is paid
    # once per B frames
    # (ipc: a frame's put is one copy issued right after its render, no batching)
    B = max(1, args.gather_batch) if ((use_dist and not ipc) or args.local_batch) else 1
    # default frames per launch (profiles/archive/r05.tar.gz: r05/ab/frames_per_launch_ab.log): depth 1: 4 (C3 0.298 ms at 4,
    # 0.300 at 8); the wavefront mode: 8 (C5 0.796 ms at 8, 0.802 at 4, 0.838 at 1)
    # (a wavefront batch's frames sit `cap` pixels apart in the rank's buffers, every rank alike: a rank
    # with fewer bands than rank 0 keeps the slot size; since round 6 the batch takes such a stride)
    wf_batch = depth > 1 and bool(flags & 8)
    FPL = args.frames_per_launch if args.frames_per_launch > 0 else (4 if depth == 1 else 8 if wf_batch else 1)
    if FPL > 1:   # a batch = the frames of one rt_render_device_batch launch (and of one gather at N > 1)
        if depth < 1 or (depth > 1 and not wf_batch) or FPL > rtamd.RT_MAX_BATCH:
            raise SystemExit(f"bench.py: --frames-per-launch needs depth 1 or the wavefront mode "
                             f"and K <= {rtamd.RT_MAX_BATCH}")
        B = FPL
    # buffer sets: batch i uses set i % NB.  At N > 1 the sets cycle 2F ways, so a batch never
    # renders into a set whose gather was issued less than F batches earlier: the gathers run
    # in issue order on one RCCL stream (the process group's, or the rt_comm's), and a render
    # waiting on the latest one would tie the streams into lock-step.  Rank 0 assembles on a
    # stream of its own.
    NB = 2 * F if use_dist else F
    streams = [torch.cuda.Stream(dev) for _ in range(F)]
    torch.cuda.set_stream(streams[0])
    outs = [torch.zeros(B, cap, dtype=torch.int32, device=dev) for _ in range(NB)]
    # rank 0: per buffer set one contiguous (world, B * cap) gather target, re-interleaved
    # into the set's B framebuffers by one rt_assemble_bands_batch launch
    gbufs = [torch.zeros(shard_n, B * cap, dtype=torch.int32, device=dev) for _ in range(NB)] \
        if (use_dist and rank == 0 and not ipc) else None
    glists = [list(g.unbind(0))[:world] for g in gbufs] if gbufs is not None else [None] * NB
    # rank 0's frames.  On the ipc path they are followed, in the same allocation, by the
    # frame-sync block (rt_frame_sync_words) that the ranks' puts and rank 0's presents share,
    # and that allocation is uncached device memory (rt_shared_alloc): peers write it over
    # xGMI while rank 0's kernels poll and read it.  Other paths: a torch tensor.
    nfr_words = NB * B * h * w
    # one completion set per frame buffer (buffer set j, frame s of its batch: q = j * B + s), so a
    # frame's put waits only for the previous use of ITS buffer -- never for the present of another
    # frame of the same batch (with B > 1 that would chain a batch's frames across ranks, and the
    # puts waiting on it spin on the GPU)
    NQ = NB * B
    sync_words = rtamd.frame_sync_words(NQ, shard_n) if ipc else 0
    shm = None

    def torch_frames():
        t = torch.zeros(nfr_words, dtype=torch.int32, device=dev)
        return list(t.view(NB, B, h * w))
    frames = torch_frames() if (rank == 0 and use_dist and not ipc) else None
    shared = None
    fsync = None
    exchange_fallback = None

    def drop_ipc():
        """Every rank leaves the IPC band puts for the torch.distributed gather (B stays 1)."""
        nonlocal ipc, tgather, shared, shm, fsync, frames, gbufs, glists
        ipc, tgather, fsync = False, True, None
        _SYNC.clear()
        if shared is not None:
            shared.close()
            shared = None
        dist.barrier()   # every peer has unmapped rank 0's frames before rank 0 frees them
        if rank == 0:
            if shm is not None:
                shm.close()
                shm = None
            frames = torch_frames()
            gbufs = [torch.zeros(shard_n, B * cap, dtype=torch.int32, device=dev) for _ in range(NB)]
            glists = [list(g.unbind(0))[:world] for g in gbufs]
    if ipc:
        # rank 0's framebuffers (+ sync block) mapped into every rank (rt_ipc_export /
        # rt_ipc_open): each rank's bands go straight to their rows of rank 0's frame.  Only
        # where every rank can reach rank 0's GPU (rt_peer_access); otherwise, or if any rank
        # cannot map them, every rank falls back to the torch.distributed gather.
        store = dist.distributed_c10d._get_default_store()
        ok = 1.0
        setup_fault = args.inject_fault if (rank == world - 1 and world > 1) else "none"
        try:
            if rank == 0:
                try:
                    shm = rtamd.SharedAlloc(local, 4 * (nfr_words + sync_words))
                    hnd, off = rtamd.SharedFrames.export(local, shm.ptr)
                    store.set("rtamd_ipc", hnd + off.to_bytes(8, "little") + local.to_bytes(4, "little"))
                except rtamd.RtError:
                    store.set("rtamd_ipc", b"")
                    raise
                fr_base = shm.ptr
            else:
                blob = bytes(store.get("rtamd_ipc"))
                if len(blob) != rtamd.SharedFrames.HANDLE_BYTES + 12:
                    raise rtamd.RtError(-2, "rank 0 could not export its frames")
                dev0 = int.from_bytes(blob[-4:], "little")
                if not rtamd.peer_access(local, dev0) or setup_fault == "no-peer":
                    raise rtamd.RtError(-2, f"device {local} cannot access rank 0's device {dev0} (no peer access"
                                            + (", injected" if setup_fault == "no-peer" else "") + ")")
                handle = blob[:-12]
                if setup_fault == "open-fails":   # a handle naming no allocation: hipIpcOpenMemHandle fails
                    handle = bytes(len(handle))
                shared = rtamd.SharedFrames.open(local, handle, int.from_bytes(blob[-12:-4], "little"))
                fr_base = shared.ptr
        except rtamd.RtError as e:
            print(f"rank {rank}: frame mapping unavailable ({e}); using torch.distributed", file=sys.stderr)
            ok = 0.0
        flag = torch.tensor([ok], device=dev)
        allreduce(flag, dist.ReduceOp.MIN)
        if flag.item() < 1.0:   # (B stays 1)
            exchange_fallback = "frame mapping unavailable on some rank"
            drop_ipc()
        else:
            put_dst = [[fr_base + 4 * (j * B + s) * h * w for s in range(B)] for j in range(NB)]
            sync_local = torch.zeros(NQ, dtype=torch.int32, device=dev)   # this rank's per-set block counters
            fsync = rtamd.FrameSync(w, h, tiling, shard_n, NQ, fr_base + 4 * nfr_words, sync_local.data_ptr(),
                                    args.sync_timeout_ms)
            _SYNC[:] = [fsync]
            if args.shard:   # the N-1 shards no process puts: their arrivals never hold the present up
                a0 = nfr_words + sync_words - NQ * shard_n   # arrive[set][rank] ends the block
                arrive = torch.full((NQ, shard_n), -1, dtype=torch.int32, device=dev)   # 0xFFFFFFFF >= every use
                arrive[:, 0] = 0
                rtamd.copy_device(fr_base + 4 * a0, arrive.data_ptr(), arrive.numel() * 4, streams[0].cuda_stream)
                torch.cuda.synchronize(dev)
            use = [0] * NQ   # times frame buffer q has been filled
    # frame checks: the camera index of every frame a set last held, and (--frame-check
    # every, rank 0) each presented frame's checksum, taken on its stream right after the
    # present saw it complete
    frame_of = [[-1] * B for _ in range(NB)]
    # the per-frame faults of the last rank (the set-up faults act elsewhere)
    fault = args.inject_fault in ("wrong-bands", "drop-put", "drop-put-warmup") and rank == world - 1 and world > 1
    fault_frame = 1 if args.inject_fault == "drop-put-warmup" else 4
    check_every = use_dist and rank == 0 and args.frame_check == "every"
    sums = torch.zeros(nframes + args.max_extra_warmup, dtype=torch.int64, device=dev) if check_every else None
    sums_ptr = sums.data_ptr() if sums is not None else 0
    checksummed = []   # frame indices whose checksum was taken at their present (ipc exchange only)

    # rays traced by this rank in a frame with params p (counted with the aux planes, untimed)
    d = max(depth, 1)
    hits = torch.zeros(npx * d * 2, dtype=torch.int32, device=dev)
    tt = torch.zeros(npx * d, dtype=torch.float32, device=dev)
    rgb = torch.zeros(npx * 3, dtype=torch.float32, device=dev)

    def count_rays(p):
        r.set_params(p)
        r.render_device(w, h, depth, flags, outs[0].data_ptr(), tiling=tiling, stream=streams[0].cuda_stream,
                        aux_ptrs=(hits.data_ptr(), tt.data_ptr(), rgb.data_ptr()))
        torch.cuda.synchronize(dev)
        hv = hits.view(npx, d, 2)
        return int((hv != -2).sum().item()), int((hv[:, 0, 0] != -2).sum().item())

    rays_f0, prim_f0 = count_rays(ptab[0])
    ray_cache = {0: (rays_f0, prim_f0)}

    def rays_of(cam):   # (rays, primary rays) of camera index cam, counted once
        if cam not in ray_cache:
            ray_cache[cam] = count_rays(ptab[cam])
        return ray_cache[cam]

    # rank 0's frame checks: its own one-rank render of a camera, and every frame a buffer set
    # holds against it (under --orbit every frame differs, so a band in the wrong frame shows)
    L = ptab.shape[0]
    sum_of = {}
    if use_dist and rank == 0 and not args.shard:
        full = torch.zeros(h * w, dtype=torch.int32, device=dev)
        ref_sum = torch.zeros(1, dtype=torch.int64, device=dev)
        got_frame = torch.zeros(h * w, dtype=torch.int32, device=dev)

    def reference(cam):   # rank 0's one-rank frame of camera index cam into `full`; its checksum
        r.set_params(ptab[cam])
        r.render_device(w, h, depth, flags, full.data_ptr(), stream=streams[0].cuda_stream)
        ref_sum.zero_()
        rtamd.frame_checksum(full.data_ptr(), h * w, ref_sum.data_ptr(), streams[0].cuda_stream)
        torch.cuda.synchronize(dev)
        sum_of[cam] = int(ref_sum.item())
        return sum_of[cam]

    held_bad = []   # frame indices of held frames that differ (diagnostics)

    def check_held():
        """(frames held, all equal): the frames rank 0's buffer sets hold vs reference()."""
        torch.cuda.synchronize(dev)
        held = [(j, s) for j in range(NB) for s in range(filled[j]) if frame_of[j][s] >= 0]
        ok = bool(held)
        held_bad.clear()
        for j, s in held:
            reference(frame_of[j][s] % L)
            if ipc:   # the uncached shared frame, copied out
                rtamd.copy_device(got_frame.data_ptr(), put_dst[j][s], 4 * h * w, streams[0].cuda_stream)
                torch.cuda.synchronize(dev)
                got = got_frame
            else:
                got = frames[j][s]
            same = bool(torch.equal(full, got))
            if not same:
                held_bad.append({"frame": frame_of[j][s], "set": j, "slot": s,
                                 "pixels_differ": int((full != got).sum().item())})
            ok = ok and same
        return len(held), ok

    # One step = one frame: render this rank's bands -> (N > 1) RCCL gather of the bands to
    # rank 0 -> rank 0 re-interleaves them into the frame.
    pending = [None] * NB     # torch path: the gather work of set j's last batch
    filled = [0] * NB         # frames in set j's last batch
    asm_used = [False] * NB
    cur = [0, 0]              # (batch number, frames rendered in it)
    nstep = [0]
    # the per-frame host path, with everything constant bound once: at N = 8 a frame is
    # ~0.05 ms of GPU time, so the host's enqueue per frame has to stay well under that
    launch = r.frame_launcher(w, h, depth, flags, tiling)
    blaunch = r.batch_launcher(w, h, depth, flags, tiling) if FPL > 1 else None
    bcams = (rtamd.rt_params * B)() if FPL > 1 else None
    base_params = rtamd.array_to_params(ptab[0])
    sh = [st.cuda_stream for st in streams]
    out_ptr = [[o[s].data_ptr() for s in range(B)] for o in outs]
    outs_ptr = [o.data_ptr() for o in outs]
    # per-frame cameras (orbit, or the jittered copies of the static camera): frame n has camera n % L
    orbit_params = [rtamd.array_to_params(p) for p in ptab] if ptab.shape[0] > 1 else None
    set_params = rtamd.lib().rt_set_params
    hdl = r._h
    if native:
        slots_ptr = [g.data_ptr() for g in gbufs] if rank == 0 else [0] * NB
        fr_ptr = [f.data_ptr() for f in frames] if rank == 0 else [0] * NB
        # (--shard: the one-rank communicator assembles this rank's own bands only)
        slot_wait, xchg = comms[0].frame_exchanger(cap, w, cap // w if args.shard else h, args.band_rows)
    pg = gopts = g_out = g_in = assemble = frame_ptr = gbuf_ptr = asm_stream = asm_sh = asm_done = gathered = None

    def torch_gather_state():
        nonlocal pg, gopts, g_out, g_in, assemble, frame_ptr, gbuf_ptr, asm_stream, asm_sh, asm_done, gathered
        pg = dist.distributed_c10d._get_default_group()
        gopts = dist.GatherOptions()
        gopts.rootRank = 0
        gopts.asyncOp = True
        g_out = [[glists[j]] if rank == 0 else [] for j in range(NB)]
        g_in = [[o.view(-1)] for o in outs]
        if rank == 0:
            assemble = rtamd.bands_assembler(w, h, shard_n, args.band_rows, B * cap, cap)
            frame_ptr = [f.data_ptr() for f in frames]
            gbuf_ptr = [g.data_ptr() for g in gbufs]
            asm_stream = torch.cuda.Stream(dev)
            asm_sh = asm_stream.cuda_stream
            asm_done = [torch.cuda.Event() for _ in range(NB)]
            gathered = [torch.cuda.Event() for _ in range(NB)]
    if tgather:
        torch_gather_state()

    def exchange(j, k, nfr):
        """Set j's batch (nfr frames, rendered on stream k = the current stream) to rank 0."""
        filled[j] = nfr
        if ipc:      # this rank's bands into their rows of rank 0's frame, after the render;
            # rank 0 then waits (on this stream) until every rank's rows of the frame are in
            for s in range(nfr):
                q = j * B + s
                src = out_ptr[j][s]
                if fault and frame_of[j][s] == fault_frame:
                    if args.inject_fault.startswith("drop-put"):
                        use[q] += 1
                        continue
                    src = out_ptr[(j + 1) % NB][s]   # another frame's bands
                fsync.put(q, use[q], src, put_dst[j][s], sh[k])
                if rank == 0:   # the set goes back to the ranks after its consumer (the checksum)
                    fsync.present(q, use[q], sh[k], release=not check_every)
                    if check_every:
                        n = frame_of[j][s]
                        if n < sums.numel():
                            rtamd.frame_checksum(put_dst[j][s], h * w, sums_ptr + 8 * n, sh[k])
                            checksummed.append(n)
                        fsync.release(q, use[q], sh[k])
                use[q] += 1
            return
        if native:   # gather on the rt_comm's stream after the renders, rank 0's assembly after it
            xchg(j, nfr, outs_ptr[j], slots_ptr[j], fr_ptr[j], sh[k])
            return
        # dist.gather(outs[j], glists[j], dst=0, async_op=True) without its argument checks,
        # then rank 0 assembles the frames on its assembly stream
        if rank == 0 and asm_used[j]:   # the set's previous assembly has read gbufs[j]
            streams[k].wait_event(asm_done[j])
        work = pg.gather(g_out[j], g_in[j], gopts)
        pending[j] = work
        if rank == 0:
            # the assembly after the gather: work.wait() orders it after the collective's own stream,
            # and the event after whatever the gather enqueued on the current stream (a one-rank group
            # may copy there instead: with distinct frames every frame, the assembly then read the set's
            # previous contents 1 run in 6 -- profiles/r06/repro_dist_check/)
            gathered[j].record(streams[k])
            torch.cuda.set_stream(asm_stream)
            asm_stream.wait_event(gathered[j])
            work.wait()   # the assembly stream after the gather
            assemble(frame_ptr[j], gbuf_ptr[j], asm_sh, nfr)
            asm_done[j].record(asm_stream)
            asm_used[j] = True
            torch.cuda.set_stream(streams[k])

    def step():
        n = nstep[0]
        nstep[0] += 1
        b, s = cur
        k, j = b % F, b % NB
        if s == 0:
            torch.cuda.set_stream(streams[k])
            if pending[j] is not None:   # set j's last gather (NB batches ago) has read outs[j]
                pending[j].wait()
                pending[j] = None
            elif native:                 # likewise, through the rt_comm's events
                slot_wait(j, sh[k])
        if FPL > 1:   # the batch's cameras; one launch renders them all when the batch is full
            bcams[s] = orbit_params[n % len(orbit_params)] if orbit_params is not None else base_params
        else:
            if orbit_params is not None:   # updateCamera (RayTracer.cpp:609-672) for this frame
                set_params(hdl, orbit_params[n % len(orbit_params)])
            launch(out_ptr[j][s], sh[k])
        frame_of[j][s] = n
        s += 1
        if s < B:
            cur[1] = s
            return
        if FPL > 1:
            blaunch(bcams, B, out_ptr[j][0], cap, sh[k])
        if use_dist:
            exchange(j, k, B)
        else:
            filled[j] = B
        cur[0], cur[1] = b + 1, 0

    def drain():
        """Send a part-filled batch as it is; the caller then synchronises the device."""
        b, s = cur
        if s and FPL > 1:   # the part-filled batch's frames, in one launch of s frames
            blaunch(bcams, s, out_ptr[b % NB][0], cap, sh[b % F])
            if not use_dist:
                filled[b % NB] = s
        if s and use_dist:
            exchange(b % NB, b % F, s)
        cur[0], cur[1] = b + (1 if s else 0), 0

    # Warm-up: the --warmup frames, then more until --warmup-seconds of frames have run (the
    # GPU's clocks ramp up over a fraction of a second after the idle scene setup: 20 frames
    # measured right after 5 warm-up frames ran 10 % slower than in steady state).  Every rank
    # warms up as many frames as the slowest-to-warm rank (agreed through an all-reduce, so the
    # ranks' frame sequences stay in step).  The ranks start it together: rank 0's present of the
    # first frame waits (bounded by --sync-timeout-ms) for every rank's first put, so a rank still
    # finishing its set-up must not eat into that bound.
    torch.cuda.synchronize(dev)
    if args.inject_fault == "slow-setup" and rank == world - 1 and world > 1:
        time.sleep(args.slow_setup_s)   # a late rank (set-up slower than the exchange bound)
    setup_skew = None
    if use_dist:
        # when this rank finished its set-up (wall clock of the one host), through the store so that
        # publishing it synchronises nothing; rank 0 reads every rank's at the end: how far apart
        # the ranks were, i.e. what the barrier below absorbs and what the first frame's bounded
        # wait would otherwise see
        dist.distributed_c10d._get_default_store().set(f"rtamd_ready_{rank}", repr(time.time()))
        if not args.no_setup_barrier:
            dist.barrier()
    for _ in range(args.warmup):
        step()
    drain()
    torch.cuda.synchronize(dev)
    tw = time.perf_counter()
    extra = 0
    while args.warmup_seconds > 0 and extra < args.max_extra_warmup:
        chunk = min(64, args.max_extra_warmup - extra)
        for _ in range(chunk):
            step()
        drain()
        torch.cuda.synchronize(dev)
        extra += chunk
        if time.perf_counter() - tw >= args.warmup_seconds:
            break
    if use_dist:   # every rank runs the largest extra warm-up of any rank
        ex = torch.tensor([float(extra)], device=dev)
        allreduce(ex, dist.ReduceOp.MAX)
        for _ in range(int(ex.item()) - extra):
            step()
        extra = int(ex.item())
        drain()
    warmup_frames = args.warmup + extra
    torch.cuda.synchronize(dev)
    # Warm-up check of the IPC exchange (N > 1): rank 0 saw every warm-up frame complete and
    # the frames it holds equal its own one-rank renders.  If not (a peer path the one-GPU
    # tests cannot exercise), every rank moves to the torch.distributed gather and warms up
    # again, and the JSON names why (`band_exchange_fallback`).  Not under the timed-region
    # faults of --inject-fault, which must surface.
    if ipc and not args.shard and args.inject_fault in ("none", "drop-put-warmup", "slow-setup"):
        ok, why = 1.0, "a rank could not take part"
        if rank == 0:
            st, presented = fsync.status()
            if st != 0 or presented != nstep[0]:
                ok, why = 0.0, f"warm-up frame delivery: status {st}, {presented} of {nstep[0]} frames presented"
            elif not check_held()[1]:
                ok, why = 0.0, "a warm-up frame differs from rank 0's one-rank render"
            r.set_params(ptab[0])
        flag = torch.tensor([ok], device=dev)
        allreduce(flag, dist.ReduceOp.MIN)
        if flag.item() < 1.0:
            exchange_fallback = why if rank == 0 else "rank 0 found the warm-up exchange failed"
            print(f"rank {rank}: IPC band exchange failed its warm-up check ({exchange_fallback}); "
                  "using torch.distributed", file=sys.stderr)
            torch.cuda.synchronize(dev)
            drop_ipc()
            torch_gather_state()
            pending[:] = [None] * NB
            filled[:] = [0] * NB
            asm_used[:] = [False] * NB
            for fo in frame_of:
                fo[:] = [-1] * B
            checksummed.clear()   # the failed IPC warm-up's checksums are not frames of this run's check
            for _ in range(args.warmup):
                step()
            drain()
            warmup_frames += args.warmup
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

    # per-launch kernel times of the timed steps, from the HIP events the library
    # records on the launch stream around each frame's kernels (ring of 64 frames)
    frame_ms_avg, kernel_ms_avg = r.timing_average(min(args.steps, 64))

    # --frames-per-launch at N = 1 (untimed, before anything else renders into the buffer sets):
    # every frame they hold, rendered by a batch launch, equals a single rt_render_device frame
    # of its camera
    batch_check = None
    if FPL > 1 and not use_dist:
        torch.cuda.synchronize(dev)
        one = torch.zeros(cap, dtype=torch.int32, device=dev)
        n_checked, batch_ok = 0, True
        for j in range(NB):
            for s_ in range(filled[j]):
                if frame_of[j][s_] < 0:
                    continue
                r.set_params(ptab[frame_of[j][s_] % ptab.shape[0]])
                r.render_device(w, h, depth, flags, one.data_ptr(), tiling=tiling, stream=streams[0].cuda_stream)
                torch.cuda.synchronize(dev)
                n_checked += 1
                batch_ok = batch_ok and bool(torch.equal(one[:npx], outs[j][s_][:npx]))
        r.set_params(ptab[0])
        batch_check = {"frames_checked": n_checked, "equal_to_single_renders": batch_ok}

    # (untimed for `value`) the same frames one per launch (rt_render_device: what a caller that has
    # only one frame at a time to give can get with F frames in flight), same cameras, same streams
    one_per_launch = None
    if FPL > 1 and not use_dist and not args.shard:
        nf = max(args.steps, 64)
        for cam in {i % L for i in range(32, nf + 32)}:
            rays_of(cam)   # counted before the timed frames
        torch.cuda.synchronize(dev)
        t1 = 0.0
        rays1 = 0
        for i in range(nf + 32):
            if i == 32:
                torch.cuda.synchronize(dev)
                t1 = time.perf_counter()
            if orbit_params is not None:
                set_params(hdl, orbit_params[i % len(orbit_params)])
            launch(out_ptr[i % NB][0], sh[i % F])
            if i >= 32:
                rays1 += rays_of(i % L)[0] if L > 1 else rays_f0
        torch.cuda.synchronize(dev)
        el1 = time.perf_counter() - t1
        r.set_params(ptab[0])
        one_per_launch = {"ms_per_frame": round(el1 / nf * 1e3, 4), "mrays_per_s": round(rays1 / el1 / 1e6, 1),
                          "frames": nf, "frames_in_flight": F,
                          "how": "rt_render_device, one frame per launch, same cameras and streams (untimed for value)"}

    total_frames = warmup_frames + args.steps
    # frame n was rendered with camera n % L (the orbit table wraps when the time-based
    # warm-up ran past it; a static camera has L = 1)
    # rays of the timed frames (untimed: one aux render per distinct camera)
    if L > 1:
        rays_local = prim_local = 0
        for n in range(warmup_frames, total_frames):
            a, b = rays_of(n % L)
            rays_local += a
            prim_local += b
        r.set_params(ptab[0])
    else:
        rays_local, prim_local = rays_f0 * args.steps, prim_f0 * args.steps
    del hits, tt, rgb

    if use_dist and rank == 0:
        st_ = dist.distributed_c10d._get_default_store()
        ready = [float(bytes(st_.get(f"rtamd_ready_{q}")).decode()) for q in range(world)]
        setup_skew = round(max(ready) - min(ready), 3)

    # Frame delivery (ipc): rank 0 observed every frame complete (rt_frame_present), or the run
    # failed.  `value` counts only presented frames.
    sync_info = None
    if fsync is not None and rank == 0:
        st, presented = fsync.status()
        sync_info = {"status": st, "frames_presented": presented, "frames_rendered": total_frames}
        if st != 0 or presented != total_frames:
            raise SystemExit(f"bench.py: frame delivery failed: {sync_info} (1 = a put timed out waiting for "
                             "its frame set, 2 = rank 0 timed out waiting for the ranks' rows)")

    # check (untimed): every frame rank 0 holds at the end (and, with --frame-check every, the
    # checksum every presented frame had when rank 0 saw it complete) equals rank 0's own
    # one-rank render of that frame's camera.  Under --orbit every frame differs, so a band
    # landing in the wrong frame, or overwriting a frame before it was presented, is caught.
    frame_ok = None
    frame_check = None
    if use_dist and rank == 0 and not args.shard:
        held, frame_ok = check_held()
        frame_check = {"held_frames_checked": held, "held_frames_equal": frame_ok,
                       "distinct_cameras": min(L, total_frames)}
        if check_every and sums is not None:
            # only the frames presented over IPC carry a checksum (after a fall-back to the RCCL
            # gather no further checksums are taken)
            got = sums.cpu().numpy()
            bad = [n for n in checksummed if int(got[n]) != sum_of.get(n % L, None) and
                   int(got[n]) != reference(n % L)]
            frame_check.update({"presented_frames_checksummed": len(checksummed), "checksum_mismatches": len(bad),
                                "mismatched_frames": bad[:16]})
            frame_ok = frame_ok and not bad
        if held_bad:
            frame_check["held_frames_differing"] = held_bad[:16]
        r.set_params(ptab[0])


    # (untimed for `value`) the reference's own boundary: rt_render, synchronous, the frame
    # read back into host memory (raytrace_gpgpu: launch + clFinish + clEnqueueReadBuffer,
    # RayTracer.cpp:330-344); pageable numpy and pinned host buffers
    # (untimed for `value`) one frame in flight: each frame's kernels from launch to completion,
    # nothing overlapping it -- the frame's critical path, which the frames in flight of the
    # timed region hide (C2: 0.25 ms alone against 0.08 ms per frame with four in flight)
    frame_latency = None
    if world == 1 and not args.shard:
        lat = []
        for _ in range(21):
            t1 = time.perf_counter()
            launch(out_ptr[0][0], sh[0])
            torch.cuda.synchronize(dev)
            lat.append((time.perf_counter() - t1) * 1e3)
        lat = sorted(lat[1:])
        frame_latency = {"ms_per_frame_median": round(lat[len(lat) // 2], 4), "ms_per_frame_min": round(lat[0], 4),
                         "ms_per_frame_mean": round(sum(lat) / len(lat), 4), "ms_per_frame_max": round(lat[-1], 4),
                         "frames": len(lat), "how": "one frame at a time: launch + device synchronize, host clock"}
        if orbit_params is not None:
            set_params(hdl, orbit_params[0])

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
                         "mrays_per_s_pinned": round(rays_f0 / (ms_pin * 1e-3) / 1e6, 1)}

    if use_dist:
        t = torch.tensor([elapsed, float(rays_local), float(prim_local)], dtype=torch.float64, device=dev)
        tmax = t[:1].clone()
        allreduce(tmax, dist.ReduceOp.MAX)
        tsum = t[1:].clone()
        allreduce(tsum, dist.ReduceOp.SUM)
        elapsed = float(tmax.item())
        rays_total, prim_total = float(tsum[0].item()), float(tsum[1].item())
        km = torch.tensor([kernel_ms_avg], dtype=torch.float64, device=dev)
        allreduce(km, dist.ReduceOp.MAX)
        kernel_ms_avg = float(km.item())
    else:
        rays_total, prim_total = float(rays_local), float(prim_local)

    ms_per_step = elapsed / args.steps * 1e3
    value = rays_total / elapsed / 1e6

    if rank != 0:
        if shared is not None:   # unmapped before rank 0 may free its frames
            shared.close()
        if world > 1:
            dist.barrier()
            for c in comms:
                c.close()
            dist.destroy_process_group()
        return

    # ---- CPU oracle leg (rank 0): algorithmic record fetches per frame (roofline), the CPU
    # baseline, and the parity check of an S_strict GPU frame against the oracle's ----
    from oracle import oracle
    scene = rtamd.Scene.from_mesh(mesh, bvh)
    cpu = None
    parity = None
    budget = args.cpu_seconds if (world == 1 and not args.no_cpu_baseline) else min(args.cpu_seconds, 5.0)
    ncores = host_threads
    tprobe = time.perf_counter()
    probe = oracle.render(scene, ptab[0], w, h, depth=depth, flags=flags, pixels=(0, (w * h) // 4093, 4093),
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
        samp = oracle.render(scene, ptab[0], w, h, depth=depth, flags=flags, pixels=(0, npix_sample, stride),
                             nthreads=ncores, aux=False)
        reps += 1
        cpu_s = time.perf_counter() - t0
        if cpu_s >= 0.6 * budget or reps >= 1000:
            break
    st = samp["stats"]
    cpu_rays = sum(st[k]["rays"] for k in ("primary", "shadow", "secondary"))
    kinds = [k for k in ("primary", "shadow", "secondary") if st[k]["rays"]]
    # per traced ray (oracle, reference visit order): the reference layout's bytes (SURVEY.md
    # 8d) and this layout's record fetches (one 64-B inner record per inner visit, one 48-B
    # triangle record per triangle test; leaves cost none: their range is in the child ref)
    bpr = sum(80.0 * st[k]["inner"] + 16.0 * st[k]["leaf"] + 64.0 * st[k]["tris"] for k in kinds) / max(1, cpu_rays)
    rec_inner = sum(st[k]["inner"] for k in kinds) / max(1, cpu_rays)
    rec_tri = sum(st[k]["tris"] for k in kinds) / max(1, cpu_rays)
    if world == 1 and not args.no_cpu_baseline:
        cpu = {"value": cpu_rays * reps / cpu_s / 1e6, "unit": "Mrays/s", "cores": ncores, "kind": "port",
               "sample": f"oracle/rt_oracle.c on every {stride}th pixel of the same frame ({npix_sample} px, "
                         f"{cpu_rays} rays) x {reps} repetition(s), {cpu_s:.1f} s, {ncores} threads = every "
                         f"core this job may use ({cpu_share['source']}: affinity {cpu_share['affinity']} CPUs, "
                         f"cgroup quota {cpu_share['cgroup_quota']}, os.cpu_count() {cpu_share['os_cpu_count']})",
               "host_cpu_share": cpu_share}
        if stride == 1:
            # the oracle's frame against the GPU's frame in the oracle's arithmetic (S_strict),
            # whole frame, same camera; the benched arithmetic is pinned to the reference
            # kernel itself by tests/test_fullsize_gpu.py
            r.set_params(ptab[0])
            gpu = r.render(w, h, depth=depth, flags=(flags & ~2) | 64)
            parity = {"mode": "S_strict (RT_FLAG_STRICT_MATH) vs oracle/rt_oracle.c", "pixels": int(w * h),
                      "equal": bool(np.array_equal(gpu, samp["out"])),
                      "differing_pixels": int(np.sum(gpu != samp["out"]))}

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

    frame_rays = rays_total / args.steps
    frame_px = float(w * h) if not args.shard else float(npx)
    alg_bytes = frame_rays * bpr + 4.0 * frame_px            # reference-layout bytes per frame
    wavefront = depth > 1 and (flags & 8)
    ns = {0: "rtk_ref", 64: "rtk_strict", 2: "rtk_hw"}[math_flags]
    kname = (f"{ns}::first_bounce_batch_kernel<true, {'true' if depth > 1 else 'false'}>" if FPL > 1
             else f"{ns}::first_bounce_kernel<true, {'true' if depth > 1 else 'false'}, 0>" if (depth == 1 or wavefront)
             else f"{ns}::render_kernel<true>")
    # ---- roofline.  The path is a gather of 48-56 B records; its time is set by
    # the vector-memory path (TA/TD), not HBM (nodes and triangles are re-read from L1/L2/Infinity
    # Cache).  That path merges the lanes of a quad that read the same record, and a load costs
    # per distinct record per quad (scripts/gather_peak_sweep.py), so its unit of work is a quad
    # request.  achieved = the frame's quad requests, counted on the GPU while rendering this
    # frame with a counting instantiation of the same kernels (rt_fetch_counts, every launch of
    # the frame), over ms_per_step; peak = the measured rate of quad requests when every
    # lane reads a different record of an L2-resident table on every CU (rt_gather_peak).
    # Both in 64-B record slots. ----
    hbm = {"bytes_per_ray_reference_layout": round(bpr, 1),
           "achieved_gbs": round(alg_bytes / (ms_per_step * 1e-3) / 1e9, 2), "peak_gbs": HBM_PEAK_GBS,
           "note": "SURVEY 8d algorithmic bytes of the reference layout; exceeds HBM peak because the scene is "
                   "served from L1/L2/Infinity Cache"}
    roof = ft = None
    fetch_cams = [0]
    if (depth == 1 or wavefront) and not args.shard and not args.no_roofline:
        # the timed frames' cameras (orbit: up to 8 spread over the timed frames, averaged)
        timed = sorted({n % L for n in range(warmup_frames, total_frames)})
        fetch_cams = [timed[i * len(timed) // min(8, len(timed))] for i in range(min(8, len(timed)))]
        try:
            fts = []
            for cam in fetch_cams:
                r.set_params(ptab[cam])
                fts.append(r.fetch_counts(w, h, depth, flags & ~16))   # every launch of the frame, counted
            ft = {k: sum(f[k] for f in fts) / len(fts) for k in fts[0]}
        except rtamd.RtError as e:                           # e.g. a scene off the fast kernel
            print(f"fetch counts unavailable: {e}", file=sys.stderr)
            ft = None
        r.set_params(ptab[0])
    if ft is not None:
        pk_ms, pk_n = r.gather_peak(16384, 256)          # 1 MiB table: L2-resident on every XCD
        quads = ft["quad_inner"] + ft["quad_tri"]
        # every lane a distinct record: one quad request per lane; at N > 1 every GPU's path
        peak_rps = world * pk_n / (pk_ms * 1e-3)
        ach_rps = quads / (ms_per_step * 1e-3)
        roof = {"bound": "l2_gather", "unit": "GB/s",
                "achieved": round(ach_rps * 64 / 1e9, 2), "peak": round(peak_rps * 64 / 1e9, 2),
                "frac": round(ach_rps / peak_rps, 4), "traffic": None,
                "roof": "quad record requests of the frame (counted on the GPU, every launch) vs random distinct "
                        "records from an L2-resident table on every CU (rt_gather_peak)"
                        + (f", x{world} GPUs" if world > 1 else ""),
                "quad_requests_per_frame": quads, "lane_fetches_per_frame": ft["inner"] + ft["tri"],
                "lanes_per_quad_request": round((ft["inner"] + ft["tri"]) / max(1, quads), 3),
                "wave_distinct_records_per_frame": ft["distinct_inner"] + ft["distinct_tri"],
                "inner_fetches": ft["inner"], "tri_fetches": ft["tri"], "distinct_inner": ft["distinct_inner"],
                "distinct_tri": ft["distinct_tri"], "wave_iterations": ft["wave_instructions"],
                "mixed_inner_tri_iterations": ft["mixed_instructions"],
                "peak_records_per_s": round(peak_rps), "peak_ns_per_record_per_cu": None,
                "fetch_counts_cameras": len(fetch_cams)}
        cus = torch.cuda.get_device_properties(dev).multi_processor_count
        roof["peak_ns_per_record_per_cu"] = round(world * cus / peak_rps * 1e9, 3)
        # The latency roof: a traversal iteration is a dependent fetch, so a wave's
        # iterations form a chain.  rt_chase_peak times one dependent traversal-shaped iteration of a
        # wave with every wave slot of the chip (8 per SIMD) running such a chain through an L2-resident
        # table, the lanes of a quad on one chain; the frame's wave iterations spread over those slots
        # then take at least iterations / slots * that time.
        ch_iters = 512
        lat = {}
        for grp in (4, 1, 64):
            ch_ms, ch_waves = r.chase_peak(16384, ch_iters, grp)
            lat[grp] = (ch_ms / ch_iters, ch_waves)
        t_iter_ms, slots = lat[4]
        model_ms = ft["wave_instructions"] / (world * slots) * t_iter_ms
        roof["latency"] = {
            "roof": "wave iterations of the frame (counted on the GPU) / wave slots x the time of one dependent "
                    "traversal-shaped iteration at full occupancy (rt_chase_peak, quad-coherent chains, L2-resident)",
            "wave_iterations_per_frame": ft["wave_instructions"], "wave_slots": world * slots,
            "ns_per_dependent_iteration": round(t_iter_ms * 1e6, 1),
            "ns_per_dependent_iteration_lane_distinct": round(lat[1][0] * 1e6, 1),
            "ns_per_dependent_iteration_wave_uniform": round(lat[64][0] * 1e6, 1),
            "model_ms": round(model_ms, 4), "frac": round(model_ms / ms_per_step, 4)}
    if roof is None:   # the fused path, or --no-roofline: the HBM model of SURVEY 8d
        roof = {"bound": "hbm", "unit": "GB/s", "achieved": hbm["achieved_gbs"], "peak": HBM_PEAK_GBS,
                "frac": round(hbm["achieved_gbs"] / HBM_PEAK_GBS, 4), "traffic": None,
                "roof": "HBM (no fetch counts for this run)"}
    # HIP-event times of one timing entry = one launch group (FPL frames): per launch and per frame
    roof.update({"hbm": hbm, "stream_copy_gbs": round(stream_copy_gbs, 1),
                 "kernel_ms_per_launch": round(kernel_ms_avg, 4), "kernel_ms_per_frame": round(kernel_ms_avg / FPL, 4),
                 "launch_kernels_ms": round(frame_ms_avg, 4), "launches_overlap": F > 1, "kernel": kname,
                 "frames_per_launch": FPL,
                 "records_per_ray_oracle": round(rec_inner + rec_tri, 2)})
    # HBM traffic: PMC counters need rocprofv3, so they come from separate profiling runs of this
    # command (scripts/pmc_c3.sh); the newest round's file is used and labelled as such, with the
    # library build it measured -- stale if that is not the library this run loaded
    pmc_files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]", f"pmc_{args.config}.json")))
    if pmc_files and not args.orbit and not args.extra_flags:
        try:
            pj = json.load(open(pmc_files[-1]))
            lib_now = rtamd.library_digest()
            # per frame, like `achieved` (a launch of the batch kernel renders frames_per_launch frames)
            roof["traffic"] = pj.get("hbm_bytes_per_frame", pj.get("hbm_bytes_per_launch"))
            if pj.get("occupancy"):   # achieved waves per SIMD of the same kernel (PMC, separate run)
                roof["occupancy"] = dict(pj["occupancy"], file=os.path.relpath(pmc_files[-1], ROOT),
                                         stale=pj.get("library_digest") != rtamd.library_digest())
            roof["traffic_source"] = {
                "file": os.path.relpath(pmc_files[-1], ROOT),
                "how": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this command (separate runs, not this "
                       "process), FETCH_SIZE x2 per the guide",
                "library_measured": pj.get("library_digest"), "library_now": lib_now,
                "stale": pj.get("library_digest") != lib_now}
        except (OSError, ValueError):
            pass

    res = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "Mrays/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "warmup_frames_run": warmup_frames,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic",
        "config": {"workload": cfg["desc"], "config": args.config, "triangles": mesh.num_triangles,
                   "bvh_nodes": int(bvh.nodes.shape[0]), "width": w, "height": h, "depth": depth,
                   "shadow": not (flags & 1), "math": MATH[math_flags], "flags": flags,
                   "camera": (f"orbit: add_rotate({args.orbit}, 0) per frame (RayTracer.cpp:553-565)" if args.orbit
                              else f"static default camera (Camera.cpp:6-19), frame n jittered by Halton(2,3) "
                                   f"sub-pixel offset n % {L} (camera 0 unjittered)" if L > 1
                              else "static default camera (Camera.cpp:6-19), every frame identical"),
                   "batch_cameras": ("distinct" if (L >= FPL * F or FPL == 1 and L >= F) else
                                     "identical" if L == 1 else "partly repeated"),
                   "block_order": "static" if flags & 16 else "adaptive longest-first from the previous frame",
                   "rays_per_frame": round(frame_rays, 1),
                   "primary_rays_per_frame": round(prim_total / args.steps, 1),
                   "primary_mrays_per_s": round(prim_total / elapsed / 1e6, 1),
                   "mpixels_per_s": round(w * h * args.steps / elapsed / 1e6, 1),
                   "parallelism": (f"shard {args.shard} of the band split (diagnostic, no gather)" if args.shard
                                   else "one rank, whole frame" if not use_dist
                                   else f"screen bands x{world} ("
                                        + ("library RCCL gather" if native else "IPC band put" if ipc else "RCCL gather")
                                        + ")"),
                   "band_rows": args.band_rows, "frames_in_flight": F, "frames_per_gather": B,
                   "frames_per_launch": FPL, "buffer_sets": NB,
                   "band_exchange": (None if not use_dist else "rt_frame_exchange (one library RCCL communicator, gather + assembly streams)" if native
                                     else "rt_bands_put: each rank's bands copied straight into rank 0's frame "
                                          "(HIP IPC mapping, no collective)" if ipc
                                     else "torch.distributed gather (RCCL), B frames per gather, + rt_assemble_bands on rank 0's "
                                     "assembly stream"),
                   "band_exchange_fallback": exchange_fallback,
                   "setup_skew_s": setup_skew,
                   "scene_distribution": (f"rank 0 builds; {scene_bytes} B scene image broadcast over RCCL "
                                          "(rt_scene_image_pack / _load)" if world > 1 else "single rank"),
                   "scene_setup_s": round(scene_s, 3),
                   "gpu_max_hw_queues": hw_queues,
                   "host_enqueue_ms_per_step": round(host_s / args.steps * 1e3, 4),
                   "bvh": ("SplitBVHBuilder (reference SBVH, same bytes)" if args.bvh == "sbvh" else "binned SAH"),
                   "bvh_refs": int(bvh.tri_indices.size), "bvh_build_s": round(build_s, 3),
                   "scene_source": "Collada (rt_mesh_load_dae)" if (cfg.get("dae", True) and not args.direct)
                   else "in-memory generator"},
        "roofline": roof,
        "cpu_baseline": cpu,
    }
    if parity is not None:
        res["parity_vs_oracle"] = parity
    if frame_ok is not None:
        res["config"]["gathered_frame_equals_single_rank_render"] = frame_ok
        res["config"]["frame_check"] = frame_check
    if batch_check is not None:
        res["config"]["batch_check"] = batch_check
    if sync_info is not None:
        res["config"]["frame_delivery"] = dict(sync_info, protocol=(
            "rt_bands_put_sync + rt_frame_present: every rank publishes its rows of each frame with a system-scope "
            "release; rank 0's stream waits for all ranks' rows of every frame before the frame counts, and a set is "
            "refilled only after rank 0 has presented (and consumed) its previous frame"))
    if host_boundary is not None:
        res["config"]["host_boundary"] = host_boundary
    if frame_latency is not None:
        res["config"]["frame_latency"] = frame_latency
    if one_per_launch is not None:
        res["config"]["one_frame_per_launch"] = one_per_launch
    print(json.dumps(res), file=result_out or sys.stdout, flush=True)
    if batch_check is not None and not batch_check["equal_to_single_renders"]:
        raise SystemExit("bench.py: a batch-launch frame differs from its single render")
    if use_dist:
        dist.barrier()
        for c in comms:
            c.close()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
