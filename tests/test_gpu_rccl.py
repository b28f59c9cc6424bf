"""The frame gather of the multi-GPU batch mode (mvstereovision3_amd/batch.py)
through RCCL on the GPU: a one-rank "nccl" process group in a child process
(torch.distributed.run, 127.0.0.1), HIP-computed int16 maps gathered as bytes,
compared with the maps themselves and with the oracle.  (The 8-rank path is
the driver's; world_size-2 gloo runs of the same code are in
tests/test_multi_rank.py and tests/test_bench_launcher.py.)"""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import os, sys
sys.path.insert(0, os.environ["MVSV_ROOT"])
import numpy as np, torch, torch.distributed as dist
import mvstereovision3_amd as mvsv
from mvstereovision3_amd.batch import gather_frames
dist.init_process_group("nccl")
dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", 0)))
torch.cuda.set_device(dev)
m = mvsv.StereoSGBM.create(1, 64, 5, 8, 40, 1, 0, 5, 0, 0, 1)
pairs = [mvsv.synth_pair(0x5EED0000 + i, 200, 96, 1, 64) for i in range(2)]
L = torch.from_numpy(np.stack([p[0] for p in pairs])).to(dev)
R = torch.from_numpy(np.stack([p[1] for p in pairs])).to(dev)
out = torch.empty((2, 96, 200), dtype=torch.int16, device=dev)
m.compute(L, R, out)
got = gather_frames(out, dist.get_rank(), dist.get_world_size(), collective=True)
torch.cuda.synchronize()
assert len(got) == 1 and got[0].dtype == torch.int16 and got[0].shape == out.shape
assert torch.equal(got[0], out), "gathered maps differ"
np.save(os.environ["MVSV_OUT"], got[0].cpu().numpy())
dist.destroy_process_group()
print("rccl gather ok")
'''


def test_rccl_gather_one_rank(gpu, mvsv, oracle, tmp_path):
    script = tmp_path / "child.py"
    script.write_text(CHILD)
    outf = tmp_path / "maps.npy"
    env = dict(os.environ, MVSV_ROOT=ROOT, MVSV_OUT=str(outf), PYTHONPATH=ROOT)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", "--master-port=29631", str(script)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "rccl gather ok" in r.stdout
    import numpy as np
    maps = np.load(outf)
    p = dict(min_disparity=1, num_disparities=64, block_size=5, p1=8, p2=40, disp12_max_diff=1,
             pre_filter_cap=0, uniqueness_ratio=5, speckle_window_size=0, speckle_range=0, mode=1)
    for i in range(2):
        L, R = mvsv.synth_pair(0x5EED0000 + i, 200, 96, 1, 64)
        assert np.array_equal(maps[i], oracle.sgbm(L, R, p)), f"frame {i}"


def test_bench_force_gather_one_rank(gpu, tmp_path):
    """bench.py --force-gather: the code path of the driver's 8-GPU run (a
    torch.distributed.run child, an NCCL process group, dist.gather of the maps
    inside the timed steps, max-over-ranks wall time) on one rank, with the
    gathered frames checked against the oracle on rank 0."""
    import json
    env = dict(os.environ, PYTHONPATH=ROOT)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--force-gather",
           "--steps", "3", "--warmup", "1", "--frames", "2", "--width", "640", "--height", "480",
           "--no-cpu-baseline"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")][-1]
    res = json.loads(line)
    assert res["n_gpus"] == 1
    assert res["config"]["gather"] == "rccl"
    assert res["config"]["launch"] == "torch.distributed.run"
    assert res["parity_sample_gathered"].startswith("1/1 "), res["parity_sample_gathered"]
    assert res["value"] > 0
