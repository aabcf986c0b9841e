"""bench.py's multi-GPU frame path on one GPU, with the assembled frames checked against a
one-rank render (bench.py's `gathered_frame_equals_single_rank_render`).  Runs bench.py as
a child process on a small config (C2 scene, 1080p, a few frames):
  * one rank through every exchange -- the IPC band puts (rt_bands_put, the default), the
    torch.distributed gather (batches of B frames, a part-filled last batch), the library's
    RCCL communicator (rt_frame_exchange) -- on a one-rank RCCL process group;
  * 2 and 3 ranks sharing the GPU (a gloo process group: RCCL refuses two ranks on one
    device) through the IPC band puts: rank 0's frames mapped into the other processes,
    every rank's bands copied into them, every frame's completion observed by rank 0 --
    the driver's N > 1 code path, end to end, on an orbiting camera, with injected faults
    that the frame check and the delivery protocol must catch."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("i,extra", [(0, []), (1, ["--inflight", "1"]), (2, ["--band-rows", "16"]),
                                     (3, ["--gather", "native"]), (4, ["--gather", "native", "--inflight", "1"]),
                                     (5, ["--gather", "torch"]),
                                     (6, ["--gather", "torch", "--gather-batch", "3", "--frames-per-launch", "1"]),
                                     (7, ["--gather", "native", "--gather-batch", "3", "--frames-per-launch", "1"]),
                                     (8, ["--gather", "torch", "--inflight", "1"]),
                                     (9, ["--frames-per-launch", "1"]), (10, ["--frames-per-launch", "3"]),
                                     (11, ["--gather", "torch", "--frames-per-launch", "3"])])
def test_bench_dist_path_assembles_the_frame(i, extra):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(29611 + i))
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--dist", "--config", "c2", "--direct", "--steps", "4",
           "--warmup", "2", "--no-cpu-baseline", "--cpu-seconds", "0.5"] + extra
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=110, env=env, cwd=ROOT)
    assert p.returncode == 0, _why(p)
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1]
    res = json.loads(line)
    assert res["config"]["gathered_frame_equals_single_rank_render"] is True, res["config"].get("frame_check")
    assert res["value"] > 0 and res["n_gpus"] == 1


@pytest.mark.parametrize("gather", ["ipc", "native"])
def test_bench_dist_shard_diagnostic_completes(gather):
    """--dist --shard 0/8: rank 0's exchange work at N = 8 with one process behind it (the
    frame-sync block counts the processes that put, not the shards)."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(29631 + (gather == "native")))
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--dist", "--shard", "0/8", "--gather", gather,
           "--config", "c2", "--direct", "--steps", "8", "--warmup", "2", "--warmup-seconds", "0",
           "--no-cpu-baseline", "--sync-timeout-ms", "2000", "--hang-timeout", "100"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=110, env=env, cwd=ROOT)
    assert p.returncode == 0, _why(p)
    res = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert res["value"] > 0 and "shard 0/8" in res["config"]["parallelism"]


def _why(p):
    """The part of a failed run's stderr that says why: bench.py's own messages (its SystemExit
    lines and rank notes), the first traceback (a rank's, before the launcher's), and the tail."""
    err = p.stderr
    own = [ln for ln in err.splitlines() if "bench.py:" in ln or ln.startswith("rank ")]
    i = err.find("Traceback (most recent call last)")
    tb = err[i:i + 2500] if i >= 0 else ""
    return "\n".join(own[-20:]) + "\n--- first traceback ---\n" + tb + "\n--- tail ---\n" + err[-1500:]


def _ranks_on_one_gpu(n, extra, timeout=115):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--gather", "ipc", "--pg", "gloo",
           "--config", "c2", "--direct", "--warmup", "2", "--warmup-seconds", "0", "--no-cpu-baseline",
           "--cpu-seconds", "0.5", "--hang-timeout", "100"] + extra   # the production exchange bound (10 s)
    return subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env, cwd=ROOT)


@pytest.mark.parametrize("n,fpl", [(2, 4), (3, 4), (2, 1), (3, 1)])
def test_bench_ranks_sharing_the_gpu_assemble_the_frame(n, fpl):
    """Every frame differs (orbiting camera); rank 0 observes each frame complete
    (rt_frame_present), checksums it right then, and every checksum and every frame it holds at
    the end equal its own one-rank render of that frame's camera.  fpl: frames per launch (the
    depth-1 default 4: each rank's bands of 4 frames in one launch, then each frame's put)."""
    p = _ranks_on_one_gpu(n, ["--steps", "24", "--orbit", "0.01", "--frame-check", "every",
                              "--frames-per-launch", str(fpl)])
    assert p.returncode == 0, _why(p)
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1]
    res = json.loads(line)
    assert res["n_gpus"] == n
    assert "rt_bands_put" in res["config"]["band_exchange"]
    fd, fc = res["config"]["frame_delivery"], res["config"]["frame_check"]
    assert fd["status"] == 0 and fd["frames_presented"] == fd["frames_rendered"] == 26
    assert fc["presented_frames_checksummed"] == 26 and fc["checksum_mismatches"] == 0, fc
    # buffer sets: 2 x 4 frames in flight, each holding its last batch (fpl frames)
    assert fc["held_frames_checked"] == (8 if fpl == 1 else 26) and fc["distinct_cameras"] == 26, fc
    assert res["config"]["gathered_frame_equals_single_rank_render"] is True, fc
    assert res["config"]["setup_skew_s"] is not None and res["config"]["band_exchange_fallback"] is None
    print(f"{n} ranks: set-up skew {res['config']['setup_skew_s']} s")


def test_ranks_sharing_the_gpu_wavefront_batches_with_ragged_bands():
    """C5 (10 M tris, depth 3 wavefront, 8 frames per launch) on 2 ranks: 1080p has 135 8-row
    bands, so rank 1 holds one band fewer than rank 0 and its batch launches take frames a slot
    (rank 0's pixel count) apart -- the round-6 strided wavefront batch, with the bounce queues in
    the cross-frame order.  Every frame of an orbiting camera is checksummed when rank 0 sees it
    complete and compared with rank 0's own one-rank render."""
    p = _ranks_on_one_gpu(2, ["--config", "c5", "--steps", "16", "--orbit", "0.01", "--frame-check", "every",
                              "--hang-timeout", "250"],
                          timeout=280)
    assert p.returncode == 0, _why(p)
    res = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    cfg = res["config"]
    assert cfg["frames_per_launch"] == 8 and cfg["depth"] == 3
    assert cfg["frame_delivery"]["status"] == 0 and cfg["frame_check"]["checksum_mismatches"] == 0, cfg["frame_check"]
    assert cfg["gathered_frame_equals_single_rank_render"] is True


@pytest.mark.parametrize("barrier", [True, False])
def test_a_late_rank_at_set_up(barrier):
    """The round-4 abort's set-up hypothesis, made deterministic: the last of 3 ranks
    finishes its set-up 3 s late, past a 1.5 s exchange bound.  With the barrier before the warm-up
    (the fix) the run completes on the IPC exchange, every frame presented; without it (the
    round-4 flow, --no-setup-barrier) rank 0's bounded wait for the first frame times out, and the
    warm-up check moves every rank to the RCCL gather -- the run still completes with exit 0, so a
    late set-up was not what aborted rank 0 with status 1."""
    extra = ["--steps", "8", "--orbit", "0.01", "--frame-check", "every", "--sync-timeout-ms", "1500",
             "--inject-fault", "slow-setup", "--slow-setup-s", "3"] + ([] if barrier else ["--no-setup-barrier"])
    p = _ranks_on_one_gpu(3, extra)
    assert p.returncode == 0, _why(p)
    res = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    cfg = res["config"]
    assert cfg["setup_skew_s"] >= 2.5, cfg["setup_skew_s"]
    assert cfg["gathered_frame_equals_single_rank_render"] is True, (cfg.get("frame_check"), cfg.get("frame_delivery"),
                                                                     cfg["band_exchange_fallback"], _why(p))
    if barrier:
        assert cfg["band_exchange_fallback"] is None and "rt_bands_put" in cfg["band_exchange"]
        assert cfg["frame_delivery"]["status"] == 0
        assert cfg["frame_check"]["checksum_mismatches"] == 0
    else:
        assert "warm-up frame delivery: status 2" in cfg["band_exchange_fallback"], cfg["band_exchange_fallback"]
        assert "torch.distributed gather" in cfg["band_exchange"]


@pytest.mark.parametrize("steps,fpl", [(10, None), (40, 1)])
def test_frame_check_catches_a_band_from_another_frame(steps, fpl):
    """The last rank puts frame 4's bands from another frame's buffer: the per-frame checksum
    (orbiting camera: every frame differs) must flag exactly that frame.  With 40 steps at one
    frame per launch the bad frame's buffer has been overwritten by the end (8 frames held), so
    only the checksum can fail the run."""
    extra = ["--steps", str(steps), "--orbit", "0.01", "--frame-check", "every", "--inject-fault", "wrong-bands"]
    if fpl:
        extra += ["--frames-per-launch", str(fpl)]
    p = _ranks_on_one_gpu(2, extra)
    assert p.returncode == 0, _why(p)
    res = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    fc = res["config"]["frame_check"]
    assert fc["checksum_mismatches"] == 1 and fc["mismatched_frames"] == [4], fc
    if steps == 40:
        assert "held_frames_differing" not in fc, fc
    assert res["config"]["gathered_frame_equals_single_rank_render"] is False


def test_frame_delivery_fails_when_a_rank_drops_a_frame():
    """The last rank never puts frame 4: rank 0's present of that frame times out (bounded wait)
    and bench.py fails instead of counting the frame."""
    p = _ranks_on_one_gpu(2, ["--steps", "6", "--sync-timeout-ms", "300", "--inject-fault", "drop-put"])
    assert p.returncode != 0
    assert "frame delivery failed" in p.stderr


def test_failed_warmup_exchange_falls_back_to_the_rccl_gather():
    """The last rank never puts warm-up frame 1: the warm-up check (rank 0's delivery status
    and held frames) moves every rank to the torch.distributed gather before the timed frames,
    which then assemble correctly; the JSON names the fallback."""
    p = _ranks_on_one_gpu(2, ["--steps", "6", "--warmup", "4", "--sync-timeout-ms", "300", "--orbit", "0.01",
                              "--inject-fault", "drop-put-warmup"])
    assert p.returncode == 0, _why(p)
    res = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert "warm-up frame delivery" in res["config"]["band_exchange_fallback"]
    assert "torch.distributed gather" in res["config"]["band_exchange"]
    assert res["config"]["gathered_frame_equals_single_rank_render"] is True


@pytest.mark.parametrize("fault,why", [("no-peer", "no peer access"), ("open-fails", "hipIpcOpenMemHandle")])
def test_unmappable_frames_fall_back_to_the_rccl_gather(fault, why):
    """The set-up half of the exchange's fallback (bench.py: peer-access gate + rt_ipc_open):
    the last rank's peer-access check says no, or it maps rank 0's frames from a handle that
    names no allocation (rt_ipc_open returns an error).  Every rank must agree to use the
    torch.distributed gather, name the reason, and its frames must equal the one-rank
    renders of an orbiting camera (every frame differs)."""
    p = _ranks_on_one_gpu(2, ["--steps", "8", "--orbit", "0.01", "--inject-fault", fault])
    assert p.returncode == 0, _why(p)
    assert why in p.stderr, p.stderr[-3000:]
    res = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert res["config"]["band_exchange_fallback"] == "frame mapping unavailable on some rank"
    assert "torch.distributed gather" in res["config"]["band_exchange"]
    assert res["config"]["frame_check"]["held_frames_checked"] > 0
    assert res["config"]["gathered_frame_equals_single_rank_render"] is True
