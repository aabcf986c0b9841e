"""bench.py's multi-GPU frame path on one GPU: a one-rank RCCL process group, the async
band gather into rank 0's slots, rt_assemble_bands, four frames in flight -- the code the
driver's N = 2..8 runs execute -- with the assembled frames checked against a one-rank
render (bench.py's `gathered_frame_equals_single_rank_render`).  Runs bench.py as a child
process on a small config (C2 scene, 1080p, a few frames)."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("i,extra", [(0, []), (1, ["--inflight", "1"]), (2, ["--band-rows", "16"]),
                                     (3, ["--gather", "native"]), (4, ["--gather", "native", "--inflight", "1"])])
def test_bench_dist_path_assembles_the_frame(i, extra):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(29611 + i))
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--dist", "--config", "c2", "--direct", "--steps", "4",
           "--warmup", "2", "--no-cpu-baseline", "--cpu-seconds", "0.5"] + extra
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=110, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1]
    res = json.loads(line)
    assert res["config"]["gathered_frame_equals_single_rank_render"] is True
    assert res["value"] > 0 and res["n_gpus"] == 1
