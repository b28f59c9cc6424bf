"""bench.py launches its own ranks when --gpus N > 1 and WORLD_SIZE is unset
(the driver's `python3 bench.py --gpus 8` shape).  --dry rehearses that
launcher and the int16-as-bytes gather on CPU with gloo (trivial host compute,
no GPU): the gathered global batch must hold every rank's frames in order."""
import json
import os

import pytest
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env,
                          capture_output=True, text=True, timeout=240)


@pytest.mark.parametrize("n", [2, 4, 8])  # the driver's scaling sweep shapes (N = 1 is the GPU bench)
def test_bench_spawns_ranks_and_gathers(n):
    r = _run(["--dry", "--gpus", str(n), "--width", "96", "--height", "48", "--frames", "2",
              "--steps", "1", "--warmup", "0"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    res = json.loads(lines[0])
    assert res["n_gpus"] == n and res["global_batch"] == 2 * n and res["gather"] == "gloo"
    assert res["gathered_frames_ok"] == f"{2 * n}/{2 * n}"


def test_bench_rejects_world_size_mismatch():
    r = _run(["--dry", "--gpus", "4"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE" in r.stderr
