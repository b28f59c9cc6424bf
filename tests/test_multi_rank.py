"""world_size-2 gloo rehearsal of the frame-parallel batch mode (CPU only).

Each rank generates its own block of the global batch, computes it (here with
the CPU oracle, on the GPU box with the HIP path in bench.py) and the maps are
gathered on rank 0; the gathered batch must equal a single-process run over
all frames.  The data path has no collective besides this gather.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

W, H, F, WORLD = 96, 48, 3, 2
P = dict(min_disparity=0, num_disparities=16, block_size=5, p1=200, p2=800, disp12_max_diff=1,
         pre_filter_cap=31, uniqueness_ratio=5, speckle_window_size=20, speckle_range=2, mode=1)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, port, result_path):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    import mvstereovision3_amd as mvsv
    from mvstereovision3_amd.batch import FrameBatch, frame_seeds
    from oracle import pyoracle
    seeds = frame_seeds(rank, WORLD, F)
    pairs = [mvsv.synth_pair(s, W, H, 0, 16) for s in seeds]
    L = torch.from_numpy(np.stack([p[0] for p in pairs]))
    R = torch.from_numpy(np.stack([p[1] for p in pairs]))
    out = torch.empty((F, H, W), dtype=torch.int16)

    def compute(Lb, Rb, o):
        for i in range(Lb.shape[0]):
            o[i] = torch.from_numpy(pyoracle.sgbm(Lb[i].numpy(), Rb[i].numpy(), P))

    batch = FrameBatch(L, R, out, compute, rank, WORLD, gather=True)
    got = batch.step()
    if rank == 0:
        np.save(result_path, torch.cat(got).numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_frame_parallel_gather_matches_single_process(tmp_path):
    import mvstereovision3_amd as mvsv
    from mvstereovision3_amd.batch import frame_seeds
    from oracle import pyoracle
    pyoracle.lib()
    path = str(tmp_path / "gathered.npy")
    mp.start_processes(_worker, args=(_free_port(), path), nprocs=WORLD, join=True,
                       start_method="spawn")
    got = np.load(path)
    assert got.shape == (WORLD * F, H, W)
    seeds = [s for r in range(WORLD) for s in frame_seeds(r, WORLD, F)]
    for i, s in enumerate(seeds):
        L, R = mvsv.synth_pair(s, W, H, 0, 16)
        assert np.array_equal(got[i], pyoracle.sgbm(L, R, P)), f"frame {i}"


def test_frame_seeds_partition():
    from mvstereovision3_amd.batch import frame_seeds
    allseeds = [s for r in range(8) for s in frame_seeds(r, 8, 8)]
    assert len(set(allseeds)) == 64 and allseeds == sorted(allseeds)
    with pytest.raises(ValueError):
        frame_seeds(8, 8, 8)
