"""Parity of the HIP render path (through the C ABI) with the CPU oracle.

The oracle computes S_strict arithmetic, so every comparison with it
renders with RT_FLAG_STRICT_MATH.  Bar: hit ids bit-exact, closest-hit
t and float RGB bit-exact (the north star allows 1e-4 on RGB; the S_strict semantics
make both sides deterministic so the test demands identity and reports the 1e-4
check separately), packed pixels bit-exact.  The default arithmetic (S_ref, the
reference's own build) is pinned to the reference kernel in test_reference_pin_gpu.py;
GPU-vs-GPU comparisons here (tilings, streams, fused vs wavefront, fast vs division
slab test) run in the default mode or in all three.
"""
import numpy as np
import pytest

from conftest import golden_names, load_golden

pytestmark = pytest.mark.gpu

RGB_TOL = 1e-4  # north star tolerance on float RGB
STRICT = 64      # RT_FLAG_STRICT_MATH: the oracle's arithmetic
WAVEFRONT, WF_SORT = 8, 32   # RT_FLAG_WAVEFRONT, RT_FLAG_WF_SORT
MODES = {"ref": 0, "strict": STRICT, "hw": 2}   # default S_ref, S_strict, S_hw (RT_FLAG_HW_MATH)


def _scene(d):
    import rtamd
    return rtamd.Scene.from_arrays(d)


def _oracle(d, depth, flags=0, w=None, h=None, params=None):
    from oracle import oracle
    w = int(d["w"]) if w is None else w
    h = int(d["h"]) if h is None else h
    return oracle.render(d, d["params"] if params is None else params, w, h, depth=depth, flags=flags)


def _compare(gpu, ref, label):
    assert np.array_equal(gpu["hits"], ref["hits"]), f"{label}: hit ids differ at " \
        f"{np.argwhere(gpu['hits'] != ref['hits'])[:5].tolist()}"
    assert np.array_equal(gpu["t"].view(np.uint32), ref["t"].view(np.uint32)), f"{label}: t differs"
    assert np.max(np.abs(gpu["rgb"] - ref["rgb"])) <= RGB_TOL, f"{label}: rgb beyond 1e-4"
    assert np.array_equal(gpu["rgb"].view(np.uint32), ref["rgb"].view(np.uint32)), f"{label}: rgb not bitwise"
    assert np.array_equal(gpu["out"], ref["out"]), f"{label}: packed pixels differ"


@pytest.mark.parametrize("name", golden_names())
def test_fixture_depth3(renderer, name):
    d = load_golden(name)
    renderer.upload(_scene(d))
    renderer.set_params(d["params"])
    w, h = int(d["w"]), int(d["h"])
    gpu = renderer.render(w, h, depth=3, flags=STRICT, aux=True)
    _compare(gpu, _oracle(d, 3), name)
    plain = renderer.render(w, h, depth=3, flags=STRICT)
    assert np.array_equal(plain, gpu["out"])


@pytest.mark.parametrize("name", ["cornell12", "knot16k", "hf40k", "rand2k"])
@pytest.mark.parametrize("depth,flags", [(1, 0), (1, 1), (2, 0), (0, 0)])
def test_depth_and_flags(renderer, name, depth, flags):
    d = load_golden(name)
    renderer.upload(_scene(d))
    renderer.set_params(d["params"])
    w, h = int(d["w"]), int(d["h"])
    gpu = renderer.render(w, h, depth=depth, flags=flags | STRICT, aux=True)
    ref = _oracle(d, depth, flags)
    _compare(gpu, ref, f"{name} depth={depth} flags={flags}")


def test_odd_sizes(renderer):
    d = load_golden("knot16k")
    import rtamd
    renderer.upload(_scene(d))
    for (w, h) in [(1, 1), (17, 9), (123, 77)]:
        m = rtamd.Mesh.torus_knot(128, 64)
        p = rtamd.params_to_array(m.camera_params(w, h))
        renderer.set_params(p)
        gpu = renderer.render(w, h, depth=3, flags=STRICT, aux=True)
        _compare(gpu, _oracle(d, 3, w=w, h=h, params=p), f"{w}x{h}")


def test_render_into_pinned_and_pageable_host_memory(renderer):
    """rt_render's frame read-back lands the same pixels in pinned and pageable host memory."""
    import torch
    d = load_golden("knot16k")
    renderer.upload(_scene(d))
    renderer.set_params(d["params"])
    w, h = int(d["w"]), int(d["h"])
    ref = _oracle(d, 1)["out"]
    pageable = np.zeros(w * h, np.uint32)
    renderer.render_host_ptr(w, h, 1, STRICT, pageable.ctypes.data)
    pinned = torch.zeros(w * h, dtype=torch.int32, pin_memory=True)
    renderer.render_host_ptr(w, h, 1, STRICT, pinned.data_ptr())
    assert np.array_equal(pageable, ref)
    assert np.array_equal(pinned.numpy().view(np.uint32), ref)
    with pytest.raises(ValueError):
        renderer.render_host_ptr(w, h, 1, 0, 0)


def test_overflow_counter(renderer):
    d = load_golden("overflow_comb")
    renderer.upload(_scene(d))
    renderer.set_params(d["params"])
    before = renderer.overflow_count()
    gpu = renderer.render(int(d["w"]), int(d["h"]), depth=3, flags=STRICT, aux=True)
    ref = _oracle(d, 3)
    _compare(gpu, ref, "overflow_comb")
    assert ref["stats"]["stack_overflow"] > 0
    assert renderer.overflow_count() > before


@pytest.mark.parametrize("nranks,band_rows", [(2, 16), (3, 8), (8, 16)])
def test_band_tiling_reassembles(renderer, nranks, band_rows):
    """Each rank's bands (rt_tiling) re-interleave to the whole frame."""
    import rtamd
    import torch
    d = load_golden("hf40k")
    renderer.upload(_scene(d))
    renderer.set_params(d["params"])
    w, h = int(d["w"]), int(d["h"]) - 8  # a short last band
    full = renderer.render(w, h, depth=1)
    img = np.zeros((h, w), np.uint32)
    nbands = (h + band_rows - 1) // band_rows
    for rank in range(nranks):
        npx = rtamd.tiling_pixels(w, h, rank, nranks, band_rows)
        buf = torch.zeros(max(npx, 1), dtype=torch.int32, device="cuda")
        t = rtamd.rt_tiling(rank, nranks, band_rows, 0)
        renderer.render_device(w, h, 1, 0, buf.data_ptr(), tiling=t)   # the ctx's own stream
        torch.cuda.synchronize()
        local = buf.cpu().numpy().view(np.uint32)[:npx].reshape(-1, w)
        row = 0
        for b in range(rank, nbands, nranks):
            n = min(band_rows, h - b * band_rows)
            img[b * band_rows:b * band_rows + n] = local[row:row + n]
            row += n
    assert np.array_equal(img.reshape(-1), full)


@pytest.mark.parametrize("nranks,band_rows,w", [(1, 8, 0), (2, 16, 0), (3, 8, 0), (8, 8, 0), (5, 8, 123)])
def test_band_puts_place_every_rank_into_the_frame(renderer, nranks, band_rows, w):
    """rt_bands_put (bench.py --gather ipc): each rank's band buffer copied into its rows of
    the frame by one strided copy (+ one for a short last band) equals a one-rank render;
    pixels outside the rank's rows are untouched."""
    import rtamd
    import torch
    d = load_golden("hf40k")
    renderer.upload(_scene(d))
    renderer.set_params(d["params"])
    w = w or int(d["w"])
    h = int(d["h"]) - 3  # a short last band
    full = renderer.render(w, h, depth=1)
    side = torch.cuda.Stream()
    frame = torch.full((h * w,), -9, dtype=torch.int32, device="cuda")
    with torch.cuda.stream(side):
        s = side.cuda_stream
        for rank in range(nranks):
            t = rtamd.rt_tiling(rank, nranks, band_rows, 0)
            buf = torch.zeros(max(1, rtamd.tiling_pixels(w, h, rank, nranks, band_rows)), dtype=torch.int32,
                              device="cuda")
            renderer.render_device(w, h, 1, 0, buf.data_ptr(), tiling=t, stream=s)
            rtamd.bands_putter(w, h, t)(buf.data_ptr(), frame.data_ptr(), s)
            torch.cuda.synchronize()
            got = frame.cpu().numpy().view(np.uint32).reshape(h, w)
            mine = np.zeros(h, bool)
            for y0, n in rtamd.rank_bands(h, rank, nranks, band_rows):
                mine[y0:y0 + n] = True
            assert np.array_equal(got[mine], full.reshape(h, w)[mine])
    assert np.array_equal(frame.cpu().numpy().view(np.uint32), full)


def test_uncached_shared_frames_take_puts_and_sync(renderer):
    """rt_shared_alloc (rank 0's shared frames + sync block for the IPC exchange, uncached so
    peers' xGMI writes and rank 0's in-kernel polling are coherent across GPUs): zeroed, IPC
    exportable, and a 3-rank frame put into it with rt_bands_put_sync and presented with
    rt_frame_present equals a one-rank render; rt_copy_device copies it out."""
    import rtamd
    import torch
    d = load_golden("hf40k")
    renderer.upload(_scene(d))
    renderer.set_params(d["params"])
    w, h = int(d["w"]), int(d["h"])
    full = renderer.render(w, h, depth=1)
    nranks, nsets = 3, 2
    sync_words = rtamd.frame_sync_words(nsets, nranks)
    shm = rtamd.SharedAlloc(0, 4 * (nsets * h * w + sync_words))
    side = torch.cuda.Stream()
    s = side.cuda_stream
    out = torch.full((nsets * h * w + sync_words,), -1, dtype=torch.int32, device="cuda")
    rtamd.copy_device(out.data_ptr(), shm.ptr, out.numel() * 4, s)
    torch.cuda.synchronize()
    assert int(out.abs().sum().item()) == 0, "rt_shared_alloc memory is not zeroed"
    hnd, off = rtamd.SharedFrames.export(0, shm.ptr)
    assert len(hnd) == rtamd.SharedFrames.HANDLE_BYTES and off == 0
    d_sync = shm.ptr + 4 * nsets * h * w
    for use in range(2):   # each set filled twice: the second fill waits for the first present
        for st in range(nsets):
            for rank in range(nranks):
                t = rtamd.rt_tiling(rank, nranks, 8, 0)
                buf = torch.zeros(rtamd.tiling_pixels(w, h, rank, nranks, 8), dtype=torch.int32, device="cuda")
                local = torch.zeros(nsets, dtype=torch.int32, device="cuda")
                local[st] = use * buf.numel() // w   # this rank's block count of earlier uses
                renderer.render_device(w, h, 1, 0, buf.data_ptr(), tiling=t, stream=s)
                fs = rtamd.FrameSync(w, h, t, nranks, nsets, d_sync, local.data_ptr(), 2000)
                fs.put(st, use, buf.data_ptr(), shm.ptr + 4 * st * h * w, s)
                torch.cuda.synchronize()
            fs.present(st, use, s)
            torch.cuda.synchronize()
            assert fs.status() == (0, use * nsets + st + 1)
            got = torch.zeros(h * w, dtype=torch.int32, device="cuda")
            rtamd.copy_device(got.data_ptr(), shm.ptr + 4 * st * h * w, 4 * h * w, s)
            torch.cuda.synchronize()
            assert np.array_equal(got.cpu().numpy().view(np.uint32), full), f"set {st} use {use}"
    shm.close()


def test_batched_band_assembly(renderer):
    """rt_assemble_bands_batch: three frames (different cameras) gathered as one batch per
    rank re-interleave to the three one-rank renders."""
    import rtamd
    import torch
    d = load_golden("hf40k")
    renderer.upload(_scene(d))
    w, h, nranks, R = int(d["w"]), int(d["h"]) - 8, 3, 8
    cam_params = []
    for k in range(3):
        p = np.array(d["params"], np.float32).copy()
        p[0:3] += 0.01 * k    # nudge the camera basis (rt_params.a)
        cam_params.append(p)
    cap = (rtamd.tiling_pixels(w, h, 0, nranks, R) + 3) // 4 * 4
    side = torch.cuda.Stream()
    slots = torch.full((nranks, 3, cap), -7, dtype=torch.int32, device="cuda")
    frames = torch.full((3, h * w), -9, dtype=torch.int32, device="cuda")
    fulls = []
    with torch.cuda.stream(side):
        s = side.cuda_stream
        for k, p in enumerate(cam_params):
            renderer.set_params(p)
            fulls.append(renderer.render(w, h, depth=1))
            for rank in range(nranks):
                t = rtamd.rt_tiling(rank, nranks, R, 0)
                renderer.render_device(w, h, 1, 0, slots[rank, k].data_ptr(), tiling=t, stream=s)
        rtamd.bands_assembler(w, h, nranks, R, 3 * cap, cap)(frames.data_ptr(), slots.data_ptr(), s, 3)
    torch.cuda.synchronize()
    for k in range(3):
        assert np.array_equal(frames[k].cpu().numpy().view(np.uint32), fulls[k]), k
    assert not np.array_equal(fulls[0], fulls[2])


@pytest.mark.parametrize("nranks,band_rows,w", [(2, 16, 0), (3, 8, 0), (8, 8, 0), (5, 8, 123)])
def test_device_band_assembly(renderer, nranks, band_rows, w):
    """bench.py's multi-GPU frame path on one device: every rank's bands rendered into
    its slot of one (nranks, slot) buffer -- what the RCCL gather delivers to rank 0 --
    then rt_assemble_bands re-interleaves them; the frame equals a one-rank render.
    w = 123 takes the unaligned (4-byte) copy path."""
    import rtamd
    import torch
    d = load_golden("hf40k")
    renderer.upload(_scene(d))
    renderer.set_params(d["params"])
    w = w or int(d["w"])
    h = int(d["h"]) - 8  # a short last band
    full = renderer.render(w, h, depth=1)
    slot = rtamd.tiling_pixels(w, h, 0, nranks, band_rows)
    slot = (slot + 3) // 4 * 4
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):   # bench.py's setting: every launch on one torch side stream
        slots = torch.full((nranks, slot), -7, dtype=torch.int32, device="cuda")
        frame = torch.full((h * w,), -9, dtype=torch.int32, device="cuda")
        s = side.cuda_stream
        for rank in range(nranks):
            t = rtamd.rt_tiling(rank, nranks, band_rows, 0)
            renderer.render_device(w, h, 1, 0, slots[rank].data_ptr(), tiling=t, stream=s)
        rtamd.assemble_bands_device(frame.data_ptr(), slots.data_ptr(), slot, w, h, nranks, band_rows, s)
    torch.cuda.synchronize()
    assert np.array_equal(frame.cpu().numpy().view(np.uint32), full)
    # the numpy host restatement of the same re-interleave agrees
    host = np.zeros(w * h, np.uint32)
    rtamd.assemble_bands(host, [x.view(np.uint32) for x in slots.cpu().numpy()], w, h, band_rows)
    assert np.array_equal(host, full)
    with pytest.raises(rtamd.RtError):   # slot too small for rank 0's bands
        rtamd.assemble_bands_device(frame.data_ptr(), slots.data_ptr(), slot // 2, w, h, nranks, band_rows, s)
    with pytest.raises(ValueError):      # the null stream is refused (NULL = ctx stream in the ABI)
        rtamd.assemble_bands_device(frame.data_ptr(), slots.data_ptr(), slot, w, h, nranks, band_rows, 0)


@pytest.mark.parametrize("depth", [1, 3])
def test_frames_in_flight_on_streams(renderer, depth):
    """Frames enqueued back to back on different streams overlap on the GPU; each stream
    has its own frame scratch in the ctx (stack spill, counters, adaptive order), so every
    frame equals the synchronous render (bench.py runs 4 frames in flight)."""
    import rtamd
    import torch
    d = load_golden("hf40k")
    renderer.upload(_scene(d))
    renderer.set_params(d["params"])
    w, h = int(d["w"]), int(d["h"])
    ref = renderer.render(w, h, depth=depth)
    streams = [torch.cuda.Stream() for _ in range(3)]
    outs = [torch.full((w * h,), -3, dtype=torch.int32, device="cuda") for _ in range(6)]
    torch.cuda.synchronize()
    for i, o in enumerate(outs):   # two rounds over three streams, nothing waited for in between
        renderer.render_device(w, h, depth, 0, o.data_ptr(), stream=streams[i % 3].cuda_stream)
    torch.cuda.synchronize()
    for o in outs:
        assert np.array_equal(o.cpu().numpy().view(np.uint32), ref)
    with pytest.raises(ValueError):   # torch's default stream (handle 0) is refused
        renderer.render_device(w, h, depth, 0, outs[0].data_ptr(), stream=0)


def test_errors(renderer):
    import rtamd
    r = rtamd.Renderer(0)
    with pytest.raises(rtamd.RtError):
        r.render(16, 16, depth=1)  # no scene
    d = load_golden("cornell12")
    s = _scene(d)
    bad = rtamd.Scene.from_arrays(s.arrays())
    bad.indices = bad.indices.copy()
    bad.indices[0] = 10 ** 6
    with pytest.raises(rtamd.RtError) as e:
        r.upload(bad)
    assert e.value.code == -5
    r.upload(s)
    with pytest.raises(rtamd.RtError):
        r.render(16, 16, depth=1)  # no params
    r.set_params(d["params"])
    with pytest.raises(rtamd.RtError):
        r.render(16, 16, depth=99)
    r.close()


@pytest.mark.parametrize("mode", sorted(MODES))
@pytest.mark.parametrize("name", ["hf40k", "knot16k", "cubes2_obj", "rand3k_bigleaf"])
def test_fast_division_is_bit_identical(renderer, name, mode):
    """The fast slab quotient (Markstein's 3 ops in S_strict / S_hw, one
    multiply by the 2.5-ulp reciprocal in S_ref) against the mode's division form."""
    import rtamd
    d = load_golden(name)
    renderer.upload(_scene(d))
    renderer.set_params(d["params"])
    w, h = int(d["w"]), int(d["h"])
    fast = renderer.render(w, h, depth=3, flags=MODES[mode], aux=True)
    slow = renderer.render(w, h, depth=3, flags=MODES[mode] | rtamd.RT_FLAG_EXACT_DIV, aux=True)
    _compare(fast, slow, f"{name} {mode} fast-vs-division")


def test_tiny_coordinates_fall_back_to_division(renderer):
    """A scene with a box coordinate below 2^-66 disables the fast quotient; results still match."""
    import rtamd
    v = np.array([[-40, -10, 1e-25, 1], [40, -10, 0, 1], [0, 50, 5, 1], [-30, 0, -30, 1], [30, 0, -30, 1],
                  [0, 0, 30, 1]], np.float32)
    m = rtamd.Mesh.from_arrays(v, np.arange(6, dtype=np.int32))
    s = rtamd.Scene.from_mesh(m, m.build_bvh())
    p = rtamd.params_to_array(m.camera_params(64, 64))
    renderer.upload(s)
    renderer.set_params(p)
    gpu = renderer.render(64, 64, depth=3, flags=STRICT, aux=True)
    from oracle import oracle
    ref = oracle.render(s, p, 64, 64, depth=3)
    _compare(gpu, ref, "tiny coordinates")
    for mode in ("ref", "hw"):   # the division form is the only one that runs here
        fast = renderer.render(64, 64, depth=3, flags=MODES[mode], aux=True)
        slow = renderer.render(64, 64, depth=3, flags=MODES[mode] | rtamd.RT_FLAG_EXACT_DIV, aux=True)
        _compare(fast, slow, "tiny coordinates " + mode)


def test_zero_direction_component_pixels(renderer):
    """An axis-aligned camera gives rays with a direction component exactly 0: the fast
    kernel's quotient takes a * (1/d) = +-inf / NaN as the IEEE quotient there (pk_xdiv's
    select) instead of handing the pixel to the general kernel; the frame must match the
    oracle bit for bit."""
    import rtamd
    d = load_golden("knot16k")
    s = _scene(d)
    renderer.upload(s)
    w = h = 65  # pixel 33: xf = 32.5 / 65 = 0.5 exactly -> image_pos.x == campos.x
    p = np.zeros((8, 4), np.float32)
    p[:, 3] = 1
    p[0, :3] = [100, 0, 0]          # a
    p[1, :3] = [0, 100, 0]          # b
    p[2, :3] = [-50, -50, 120]      # c
    p[3, :3] = [0, 0, 220]          # campos
    p[4, :3] = [-23, 200, 3]
    p[5, :3] = [1, 1, 1]
    p[6, :3] = d["scene_min"]
    p[7, :3] = d["scene_max"]
    p = p.reshape(-1)
    renderer.set_params(p)
    gpu = renderer.render(w, h, depth=3, flags=STRICT, aux=True)
    _compare(gpu, _oracle(d, 3, w=w, h=h, params=p), "axis-aligned camera")
    assert renderer.last_deferred() == 0
    import rtamd
    for mode in ("ref", "hw"):   # zero components through each mode's fast quotient
        fast = renderer.render(w, h, depth=3, flags=MODES[mode], aux=True)
        slow = renderer.render(w, h, depth=3, flags=MODES[mode] | rtamd.RT_FLAG_EXACT_DIV, aux=True)
        _compare(fast, slow, "axis-aligned camera " + mode)


@pytest.mark.parametrize("name", golden_names())
@pytest.mark.parametrize("depth", [1, 3])
@pytest.mark.parametrize("sort", [False, True])
def test_wavefront_path_matches_oracle(renderer, name, depth, sort):
    """RT_FLAG_WAVEFRONT (one launch per bounce over a compacted ray queue, optionally
    sorted per bounce) against the CPU oracle directly, aux planes included."""
    import rtamd
    d = load_golden(name)
    renderer.upload(_scene(d))
    renderer.set_params(d["params"])
    w, h = int(d["w"]), int(d["h"])
    flags = STRICT | rtamd.RT_FLAG_WAVEFRONT | (rtamd.RT_FLAG_WF_SORT if sort else 0)
    ref = _oracle(d, depth)
    _compare(renderer.render(w, h, depth=depth, flags=flags, aux=True), ref, f"{name} depth={depth} sort={sort}")
    # second frame: longest-first block order from the first one's times
    _compare(renderer.render(w, h, depth=depth, flags=flags, aux=True), ref, f"{name} depth={depth} sort={sort} (2)")


def test_wavefront_frames_of_changing_depth_and_size(renderer):
    """One renderer (one stream, one frame slot) renders wavefront frames whose depth and
    size change from frame to frame: the segmented queues, their chunk sums and the frame
    counters (two parity sets, the next frame's zeroed by this one) are resized and reused;
    every frame equals the oracle's."""
    import rtamd
    d = load_golden("knot16k")
    renderer.upload(_scene(d))
    renderer.set_params(d["params"])
    w, h = int(d["w"]), int(d["h"])
    refs = {}
    seq = [(3, w, h), (1, w, h), (3, w, h), (2, w // 2, h // 2), (3, w, h), (8, w // 2 + 5, h // 2 + 3),
           (1, w // 2, h // 2), (3, w, h)]
    for i, (depth, fw, fh) in enumerate(seq):
        for sort in (False, True):
            flags = STRICT | WAVEFRONT | (WF_SORT if sort else 0)
            key = (depth, fw, fh)
            if key not in refs:
                refs[key] = _oracle(d, depth, w=fw, h=fh)
            _compare(renderer.render(fw, fh, depth=depth, flags=flags, aux=True), refs[key],
                     f"frame {i}: depth {depth} {fw}x{fh} sort={sort}")


@pytest.mark.parametrize("name", golden_names())
@pytest.mark.parametrize("depth", [1, 3])
@pytest.mark.parametrize("sort", [False, True])
def test_fused_and_wavefront_paths_agree(renderer, name, depth, sort):
    """The default fused kernel and RT_FLAG_WAVEFRONT (one launch per bounce over a compacted
    ray queue, optionally sorted per bounce) give the same bits, aux planes included."""
    import rtamd
    d = load_golden(name)
    renderer.upload(_scene(d))
    renderer.set_params(d["params"])
    w, h = int(d["w"]), int(d["h"])
    fused = renderer.render(w, h, depth=depth, aux=True)
    flags = rtamd.RT_FLAG_WAVEFRONT | (rtamd.RT_FLAG_WF_SORT if sort else 0)
    wf = renderer.render(w, h, depth=depth, flags=flags, aux=True)
    _compare(wf, fused, f"{name} depth={depth} sort={sort} wavefront-vs-fused")
    wf2 = renderer.render(w, h, depth=depth, flags=flags, aux=True)   # longest-first block order
    _compare(wf2, fused, f"{name} depth={depth} sort={sort} wavefront-vs-fused (adaptive order)")


@pytest.mark.parametrize("name", ["hf40k", "knot16k"])
def test_adaptive_block_order_is_bit_identical(renderer, name):
    """Frames after the first run blocks longest-first from the previous frame's per-tile
    times (tile_order_kernel); RT_FLAG_STATIC_ORDER keeps the static order.  Same pixels."""
    import rtamd
    d = load_golden(name)
    renderer.upload(_scene(d))
    renderer.set_params(d["params"])
    w, h = int(d["w"]), int(d["h"])
    static = renderer.render(w, h, depth=3, flags=rtamd.RT_FLAG_STATIC_ORDER | STRICT, aux=True)
    first = renderer.render(w, h, depth=3, flags=STRICT, aux=True)   # measures
    second = renderer.render(w, h, depth=3, flags=STRICT, aux=True)  # longest-first order
    _compare(first, static, name + " first adaptive frame")
    _compare(second, static, name + " adaptive order")
    _compare(second, _oracle(d, 3), name + " adaptive vs oracle")


@pytest.mark.parametrize("make", ["random_splits", "knot"])
def test_sbvh_scene_parity(renderer, make):
    """Scenes on the reference's spatial-split BVH (duplicated references, rt_bvh_build_sbvh)."""
    import rtamd
    from oracle import oracle
    m = rtamd.Mesh.random(6000, 100.0, 12.0, 3) if make == "random_splits" else rtamd.Mesh.torus_knot(96, 40)
    s = rtamd.Scene.from_mesh(m, m.build_sbvh())
    w, h = 96, 64
    p = rtamd.params_to_array(m.camera_params(w, h))
    renderer.upload(s)
    renderer.set_params(p)
    gpu = renderer.render(w, h, depth=3, flags=STRICT, aux=True)
    _compare(gpu, oracle.render(s, p, w, h, depth=3), "sbvh " + make)


def test_scene_image_moves_the_scene_between_contexts(renderer):
    """rt_scene_image_pack on one ctx + rt_scene_image_load on another (what bench.py does
    across ranks, with an RCCL broadcast of the image in between): the second ctx renders
    the same frames, in every arithmetic, without ever seeing the host arrays."""
    import rtamd
    import torch
    d = load_golden("rand4k_sbvh")
    renderer.upload(_scene(d))
    n = renderer.scene_image_size()
    img = torch.zeros(n, dtype=torch.uint8, device="cuda")
    renderer.pack_scene(img.data_ptr(), n)
    other = rtamd.Renderer(0)
    other.load_scene(img.data_ptr(), n)
    del img
    w, h = int(d["w"]), int(d["h"])
    for r in (renderer, other):
        r.set_params(d["params"])
    for flags in (0, STRICT, 2, STRICT | rtamd.RT_FLAG_WAVEFRONT | rtamd.RT_FLAG_WF_SORT):
        a = renderer.render(w, h, depth=3, flags=flags, aux=True)
        b = other.render(w, h, depth=3, flags=flags, aux=True)
        _compare(b, a, f"scene image flags={flags}")
    _compare(other.render(w, h, depth=3, flags=STRICT, aux=True), _oracle(d, 3), "scene image vs oracle")
    bad = torch.zeros(4096, dtype=torch.uint8, device="cuda")
    with pytest.raises(rtamd.RtError):
        other.load_scene(bad.data_ptr(), 4096)   # no magic: refused, the old scene stays
    _compare(other.render(w, h, depth=3, flags=STRICT, aux=True), _oracle(d, 3), "after a refused image")
    other.close()


@pytest.mark.parametrize("name", ["hf40k", "cubes2_dae"])
def test_fetch_counts_are_the_oracles_visits(renderer, name):
    """The counting instantiation behind the roofline (rt_fetch_counts): in S_strict its
    inner-record fetches are exactly the oracle's inner visits (the reference's visit order)
    and its triangle-record fetches the oracle's triangle tests (plus one per visit of an
    empty leaf) -- for a depth-1 frame (primary + shadow rays) and for a depth-3 frame on the
    wavefront path (every bounce launch, primary, shadow and secondary rays)."""
    from oracle import oracle
    d = load_golden(name)
    renderer.upload(_scene(d))
    renderer.set_params(d["params"])
    w, h = int(d["w"]), int(d["h"])
    for depth, flags in ((1, STRICT), (3, STRICT | WAVEFRONT), (3, STRICT | WAVEFRONT | WF_SORT)):
        fr = renderer.fetch_counts(w, h, depth, flags)
        assert renderer.last_deferred() == 0   # no restarted (uncounted) traversals
        assert fr["wave_instructions"] > 0 and fr["mixed_instructions"] <= fr["wave_instructions"]
        assert 0 < fr["distinct_inner"] <= fr["quad_inner"] <= fr["inner"]
        assert 0 < fr["distinct_tri"] <= fr["quad_tri"] <= fr["tri"]
        st = oracle.render(d, d["params"], w, h, depth=depth, aux=False)["stats"]
        kinds = ("primary", "shadow", "secondary")
        inner = sum(st[k]["inner"] for k in kinds)
        tris = sum(st[k]["tris"] for k in kinds)
        leaves = sum(st[k]["leaf"] for k in kinds)
        assert fr["inner"] == inner, (depth, flags)
        assert tris <= fr["tri"] <= tris + leaves, (depth, flags)
    with pytest.raises(Exception):
        renderer.fetch_counts(w, h, 3, STRICT)   # the fused path has no counting instantiation
    ms, n = renderer.gather_peak(4096, 64)
    assert ms > 0 and n > 0


@pytest.mark.parametrize("name", ["knot16k", "rand4k_sbvh"])
def test_records_beyond_the_buffer_load_limit_render_with_the_general_traversal(renderer, name, monkeypatch):
    """Scenes whose inner + triangle records reach the 31-bit buffer-load limit (2 GiB, about
    25 M triangle references) get two allocations and render with the general traversal.
    RTAMD_RECORD_LIMIT lowers the limit so a fixture takes that path: same bits as the oracle,
    in every mode, on the fused and wavefront paths, and through a scene image."""
    import rtamd
    d = load_golden(name)
    w, h = int(d["w"]), int(d["h"])
    ref = _oracle(d, 3)
    normal = {}
    renderer.upload(_scene(d))
    renderer.set_params(d["params"])
    for m, f in MODES.items():
        normal[m] = renderer.render(w, h, depth=3, flags=f)
    monkeypatch.setenv("RTAMD_RECORD_LIMIT", "1024")
    renderer.upload(_scene(d))
    renderer.set_params(d["params"])
    _compare(renderer.render(w, h, depth=3, flags=STRICT, aux=True), ref, f"{name} split records")
    for m, f in MODES.items():
        assert np.array_equal(renderer.render(w, h, depth=3, flags=f), normal[m]), m
        assert np.array_equal(renderer.render(w, h, depth=3, flags=f | WAVEFRONT), normal[m]), m
    with pytest.raises(rtamd.RtError):   # the counting kernels are fast-path only
        renderer.fetch_counts(w, h, 1, 0)
    # moved through a scene image into a second context (which allocates split records too)
    import torch
    nb = renderer.scene_image_size()
    img = torch.empty(nb, dtype=torch.uint8, device="cuda")
    renderer.pack_scene(img.data_ptr(), nb)
    r2 = rtamd.Renderer(0)
    try:
        r2.load_scene(img.data_ptr(), nb)
        r2.set_params(d["params"])
        assert np.array_equal(r2.render(w, h, depth=3, flags=0), normal["ref"])
    finally:
        r2.close()
    monkeypatch.delenv("RTAMD_RECORD_LIMIT")
    renderer.upload(_scene(d))   # back to one allocation for the tests that follow


def test_latency_and_gather_roofs_measure(renderer):
    """rt_chase_peak / rt_gather_peak return sane ceilings.  Each chain time is the minimum of
    three launch sets (clock ramp and run-to-run noise); only the wide ordering is asserted:
    lane-distinct chains (four times the quad requests) measure ~2.5x the coherent ones, while
    wave-uniform and quad-coherent chains are within noise of each other."""
    import math

    def best(group):
        runs = [renderer.chase_peak(16384, 256, group) for _ in range(3)]
        return min(r[0] for r in runs), runs[0][1]
    ms4, waves = best(4)
    ms1, _ = best(1)
    ms64, _ = best(64)
    assert waves > 0 and all(math.isfinite(m) and m > 0 for m in (ms4, ms1, ms64))
    assert ms4 <= ms1 * 1.05 and ms64 <= ms1 * 1.05
    pk_ms, pk_n = renderer.gather_peak(16384, 256)
    assert pk_ms > 0 and pk_n > 0


def test_triangle_records_beyond_2_to_the_24(renderer):
    """A leaf whose triangle records lie at index >= 2^24 of the record array: the fast
    traversal addresses them by byte offset (tk, a 32-bit byte cursor), so scenes of more than
    16.8 M triangle references render the same triangles as small ones.  The knot fixture's
    reference array gets 2^24 + 5 padding entries in front (every leaf range shifted past
    them, about 0.8 GB of triangle records, still one allocation): its depth-1 frames (the
    benched first_bounce_kernel with its offset select) and depth-3 frames equal the unpadded
    scene's in every mode, and the S_strict frame equals the oracle's."""
    d = load_golden("knot16k")
    w, h = int(d["w"]), int(d["h"])
    base = _scene(d)
    renderer.upload(base)
    renderer.set_params(d["params"])
    want = {(dep, m): renderer.render(w, h, depth=dep, flags=f, aux=True) for dep in (1, 3) for m, f in MODES.items()}
    pad = (1 << 24) + 5
    big = _scene(d)
    big.tri_indices = np.concatenate([np.full(pad, base.tri_indices[0], np.int32), base.tri_indices])
    big.nodes = big.nodes.copy()   # (from_arrays may share the fixture's arrays)
    ni = big.nodes.view(np.int32)
    leaf = ni[:, 8] < 0
    ni[leaf, 10] += pad
    renderer.upload(big)
    renderer.set_params(d["params"])
    try:
        for (dep, m), ref in want.items():
            got = renderer.render(w, h, depth=dep, flags=MODES[m], aux=True)
            _compare(got, ref, f"padded refs, depth {dep}, {m}")
        _compare(renderer.render(w, h, depth=3, flags=STRICT, aux=True), _oracle(d, 3), "padded refs vs oracle")
    finally:
        renderer.upload(base)


def test_render_readback_paths_agree(renderer):
    """rt_render (the reference's synchronous boundary, raytrace_gpgpu) on a frame large enough
    for its row groups (>= 512 x 512): into pageable memory (row groups read back while later
    groups render), into pinned host memory, with aux planes, and via rt_render_device -- the
    same pixels, and the aux planes equal a one-launch device render's."""
    import torch
    d = load_golden("knot16k")
    renderer.upload(_scene(d))
    w, h = 1024, 720
    p = d["params"].copy()
    renderer.set_params(p)
    dev = torch.zeros(w * h, dtype=torch.int32, device="cuda")
    s = torch.cuda.Stream()
    renderer.render_device(w, h, 1, 0, dev.data_ptr(), stream=s.cuda_stream)
    torch.cuda.synchronize()
    want = dev.cpu().numpy().view(np.uint32)
    pageable = np.zeros(w * h, np.uint32)
    renderer.render_host_ptr(w, h, 1, 0, pageable.ctypes.data)
    pinned = torch.zeros(w * h, dtype=torch.int32, pin_memory=True)
    renderer.render_host_ptr(w, h, 1, 0, pinned.data_ptr())
    assert np.array_equal(pageable, want)
    assert np.array_equal(pinned.numpy().view(np.uint32), want)
    for depth, flags in ((1, 0), (3, STRICT), (3, WAVEFRONT | WF_SORT)):
        a = renderer.render(w, h, depth=depth, flags=flags, aux=True)   # rt_render, row groups
        hits = torch.zeros(w * h * depth * 2, dtype=torch.int32, device="cuda")
        tt = torch.zeros(w * h * depth, dtype=torch.float32, device="cuda")
        rgb = torch.zeros(w * h * 3, dtype=torch.float32, device="cuda")
        renderer.render_device(w, h, depth, flags, dev.data_ptr(), stream=s.cuda_stream,
                               aux_ptrs=(hits.data_ptr(), tt.data_ptr(), rgb.data_ptr()))
        torch.cuda.synchronize()
        assert np.array_equal(a["out"], dev.cpu().numpy().view(np.uint32)), (depth, flags)
        assert np.array_equal(a["hits"].reshape(-1), hits.cpu().numpy()), (depth, flags)
        assert np.array_equal(a["t"].reshape(-1).view(np.uint32), tt.cpu().numpy().view(np.uint32)), (depth, flags)
        assert np.array_equal(a["rgb"].reshape(-1).view(np.uint32), rgb.cpu().numpy().view(np.uint32)), (depth, flags)


@pytest.mark.parametrize("w,h,depth,flags", [(640, 360, 1, 0), (1920, 1080, 1, 0), (3840, 2160, 1, 0),
                                             (640, 360, 3, WAVEFRONT | WF_SORT)])
def test_adaptive_order_renders_every_tile_of_a_moving_camera(renderer, w, h, depth, flags):
    """Frames of an orbiting camera rendered one after another on one stream each use the
    longest-first block order built by the stream slot's latest rebuild launch (launches 0, 8
    and 16 here: the order is rebuilt every 8th launch, the launches between have no block
    epilogue; rtk::tile_epilogue: costs read 16 per thread per round trip, bucket keys kept in
    LDS up to kKeyBytes blocks, re-read beyond: 3840x2160 has 32,400 blocks).  Every frame starts
    from a sentinel-filled buffer and must equal the static-order render of its camera: an order
    that is not a permutation of the blocks leaves sentinel pixels (a skipped tile) behind."""
    import torch
    import rtamd
    d = load_golden("knot16k")
    renderer.upload(_scene(d))
    m = rtamd.Mesh.torus_knot(128, 64)
    cam = rtamd.Camera()
    buf = torch.empty(w * h, dtype=torch.int32, device="cuda")
    s = torch.cuda.Stream()
    for f in range(18):
        cam.add_rotate(0.07, 0.0)
        renderer.set_params(rtamd.params_to_array(cam.params(m, w, h)))
        with torch.cuda.stream(s):
            buf.fill_(-1)
        renderer.render_device(w, h, depth, flags, buf.data_ptr(), stream=s.cuda_stream)
        torch.cuda.synchronize()
        got = buf.cpu().numpy().view(np.uint32)
        want = renderer.render(w, h, depth=depth, flags=flags | 16)   # RT_FLAG_STATIC_ORDER
        bad = int(np.sum(got != want))
        assert bad == 0, f"frame {f}: {bad} pixels differ ({int(np.sum(got == 0xFFFFFFFF))} sentinel)"
