"""bench.py's multi-rank entry point on the CPU: `python bench.py --gpus N` starts N ranks
through torch.distributed.run (one process per GPU in a real run), and a torchrun-launched
bench whose WORLD_SIZE disagrees with --gpus refuses to run.  --probe-launch stops each
rank after a gloo rendezvous, so no GPU is needed."""
import json
import os
import subprocess
import sys

from conftest import ROOT

BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(kw)
    return env


def test_launcher_command_is_one_node_torchrun():
    sys.path.insert(0, ROOT)
    import bench
    cmd = bench.launcher_cmd(8, ["--gpus", "8", "--steps", "5"], 29999)
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-3:] == ["--gpus", "8", "--steps", "5"] or cmd[-4:] == ["--gpus", "8", "--steps", "5"]


def test_gpus_n_launches_n_ranks():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--probe-launch"], capture_output=True, text=True,
                       timeout=180, env=_env(), cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    res = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert res["n_gpus"] == 2 and res["gpus_arg"] == 2 and res["all_reduce"] == 2.0
    assert sorted(x["rank"] for x in res["ranks"]) == [0, 1]


def test_world_size_must_match_gpus():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "1", "--probe-launch"], capture_output=True, text=True,
                       timeout=60, env=_env(WORLD_SIZE="2", RANK="0"), cwd=ROOT)
    assert p.returncode != 0 and "WORLD_SIZE=2" in p.stderr


def test_jittered_cameras_are_distinct_subpixel_shifts():
    """bench.py's default cameras: copy 0 is the camera itself, every copy differs from every other,
    and each moves the image plane by less than half a pixel along a and b (volumeRender.cl:1169-1190:
    image_pos = c + a xf + b yf, xf = (x - 0.5) / w), with the eye, light and scene box unchanged."""
    import numpy as np
    sys.path.insert(0, ROOT)
    import bench
    rng = np.random.default_rng(7)
    p = rng.normal(size=32).astype(np.float32) * 100
    w, h = 1920, 1080
    cams = bench.jittered_cameras(p, w, h, 32)
    assert cams.shape == (32, 32) and np.array_equal(cams[0], p)
    assert len({c.tobytes() for c in cams}) == 32
    a, b = p[0:3].astype(np.float64), p[4:7].astype(np.float64)
    A = np.stack([a, b], 1)
    for c in cams[1:]:
        d = c[8:11].astype(np.float64) - p[8:11].astype(np.float64)
        (dx, dy), *_ = np.linalg.lstsq(A, d, rcond=None)
        assert abs(dx * w) <= 0.5 + 1e-3 and abs(dy * h) <= 0.5 + 1e-3, (dx * w, dy * h)
        mask = np.ones(32, bool)
        mask[8:11] = False
        assert np.array_equal(c[mask], p[mask])
