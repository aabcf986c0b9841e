"""Multi-rank frame sharding on CPU (gloo, world_size 2 and 3).

Each rank owns the 16-row bands b with b % nranks == rank (rt_tiling), renders
them (here with the CPU oracle standing in for the GPU, since this runs without
one), gathers its band buffer to rank 0 with torch.distributed, and rank 0
re-interleaves them with rtamd.assemble_bands -- the exact host logic bench.py
runs over RCCL.  The assembled frame must equal a single-rank render.
"""
import os
import socket

import numpy as np
import pytest

from conftest import PKG, ROOT, load_golden


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, band_rows, q):
    import sys
    for p in (PKG, ROOT):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch
    import torch.distributed as dist
    import rtamd
    from oracle import oracle
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    d = load_golden("hf40k")
    w, h = int(d["w"]), int(d["h"]) - 8
    npx = rtamd.tiling_pixels(w, h, rank, world, band_rows)
    nbands = (h + band_rows - 1) // band_rows
    cap = ((nbands + world - 1) // world) * band_rows * w
    buf = np.zeros(cap, np.uint32)
    row = 0
    for y0, n in rtamd.rank_bands(h, rank, world, band_rows):
        r = oracle.render(d, d["params"], w, h, depth=1, pixels=(y0 * w, n * w, 1), nthreads=2, aux=False)
        buf[row * w:(row + n) * w] = r["out"]
        row += n
    assert row * w == npx
    t = torch.from_numpy(buf.view(np.int32))
    gl = [torch.zeros(cap, dtype=torch.int32) for _ in range(world)] if rank == 0 else None
    dist.gather(t, gather_list=gl, dst=0)
    if rank == 0:
        frame = np.zeros(w * h, np.uint32)
        rtamd.assemble_bands(frame, [g.numpy().view(np.uint32) for g in gl], w, h, band_rows)
        full = oracle.render(d, d["params"], w, h, depth=1, nthreads=2, aux=False)["out"]
        q.put(bool(np.array_equal(frame, full)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,band_rows", [(2, 16), (3, 8)])
def test_gloo_band_gather_reassembles_frame(world, band_rows):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, band_rows, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    assert all(p.exitcode == 0 for p in procs)
    assert q.get(timeout=10) is True


def test_rank_bands_partition():
    import rtamd
    for h in (1, 15, 16, 17, 1080, 2160):
        for n in (1, 2, 3, 8):
            rows = sorted(y for r in range(n) for (y0, k) in rtamd.rank_bands(h, r, n, 16) for y in range(y0, y0 + k))
            assert rows == list(range(h))
            for r in range(n):
                assert sum(k for _, k in rtamd.rank_bands(h, r, n, 16)) * 7 == rtamd.tiling_pixels(7, h, r, n, 16)
