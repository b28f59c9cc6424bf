"""HIP-graph replay of repeated small launches (round 6, mvsv_host.cpp graph_run;
opt-in with MVSV_GRAPHS=1 -- measured slower than eager launches on ROCm 7.2,
DESIGN.md): the first call with a set of arguments runs eagerly, its repeat is
captured, later ones launch the graph.  The replayed graph must read the
current contents of the caller's buffers, follow a reallocation of the
context's buffers (a call with another shape in between), and work from the
legacy null stream; every output bit-exact against the oracle.
Reference: Disparity::sgbm (src/disparity.cpp:6-10) called once per camera frame
on the same buffers (trgt/liveDisparity.cpp:82-101)."""
import numpy as np
import pytest

from tests.test_gpu_parity import report

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("mode", [0, 1])
def test_graph_replay_same_buffers(gpu, mvsv, oracle, mode, monkeypatch):
    torch = gpu
    monkeypatch.setenv("MVSV_GRAPHS", "1")
    from mvstereovision3_amd import _lib
    dev = torch.device("cuda", 0)
    m = mvsv.StereoSGBM.create(1, 128, 13, 0, 0, 0, 0, 0, 150, 2, mode)
    p = {k: v for k, v in m.params().items() if k != "variant"}
    frames = [mvsv.synth_pair(0x6A000000 + i, 640, 480, 1, 128) for i in range(5)]
    L = torch.empty((480, 640), dtype=torch.uint8, device=dev)
    R = torch.empty_like(L)
    out = torch.empty((480, 640), dtype=torch.int16, device=dev)
    ctx = _lib.Context(0)
    try:
        with _lib.use_context(ctx):
            for i, (Lh, Rh) in enumerate(frames + frames[:2]):
                L.copy_(torch.from_numpy(Lh))
                R.copy_(torch.from_numpy(Rh))
                m.compute(L, R, out)
                if i == 4:
                    # another shape in between: the context's buffers grow, the
                    # graph of the 640x480 call must be retired and re-captured
                    big = torch.zeros((2, 960, 1280), dtype=torch.uint8, device=dev)
                    m.compute(big, big, torch.empty((2, 960, 1280), dtype=torch.int16, device=dev))
                torch.cuda.synchronize()
                got = out.cpu().numpy()
                want = oracle.sgbm(Lh, Rh, p)
                assert np.array_equal(got, want), f"mode {mode} call {i}: " + report(got, want)
    finally:
        ctx.close()


def test_graph_replay_null_stream(gpu, mvsv, oracle, monkeypatch):
    """Host-pointer calls run on the context's own stream; device calls from
    torch's default (legacy null) stream are captured on the capture stream."""
    torch = gpu
    from mvstereovision3_amd import _lib
    monkeypatch.setenv("MVSV_GRAPHS", "1")
    ctx = _lib.Context(0)
    dev = torch.device("cuda", 0)
    m = mvsv.StereoSGBM.create(1, 128, 13, 0, 0, 0, 0, 0, 150, 2, 0)
    p = {k: v for k, v in m.params().items() if k != "variant"}
    Lh, Rh = mvsv.synth_pair(0x6A100000, 640, 480, 1, 128)
    L = torch.from_numpy(Lh).to(dev)
    R = torch.from_numpy(Rh).to(dev)
    out = torch.empty((480, 640), dtype=torch.int16, device=dev)
    want = oracle.sgbm(Lh, Rh, p)
    try:
        with _lib.use_context(ctx), torch.cuda.stream(torch.cuda.default_stream(dev)):
            for i in range(4):
                out.zero_()
                m.compute(L, R, out)
                torch.cuda.synchronize()
                assert np.array_equal(out.cpu().numpy(), want), f"call {i}"
            for i in range(3):  # host pointers (PCIe path) repeat too
                assert np.array_equal(m.compute(Lh, Rh), want), f"host call {i}"
    finally:
        ctx.close()


@pytest.mark.parametrize("cfg", ["bm_yml", "d64"])
def test_graph_replay_bm(gpu, mvsv, oracle, cfg, monkeypatch):
    """StereoBM (configs 1 and 2) repeated on the same device buffers: eager,
    captured, replayed -- every call against the oracle on fresh contents."""
    import os
    torch = gpu
    from mvstereovision3_amd import _lib
    monkeypatch.setenv("MVSV_GRAPHS", "1")
    ctx = _lib.Context(0)
    from tests.conftest import GOLDEN
    dev = torch.device("cuda", 0)
    if cfg == "bm_yml":
        b = mvsv.StereoBM.create(0, 21)
        assert mvsv.Disparity.loadBMParameters(os.path.join(GOLDEN, "configs", "bm.yml"), b)
        D = 80
    else:
        b = mvsv.StereoBM.create(64, 9)
        D = 64
    bp = b.params()
    frames = [mvsv.synth_pair(0x6A200000 + i, 640, 480, 0, D) for i in range(4)]
    L = torch.empty((2, 480, 640), dtype=torch.uint8, device=dev)
    R = torch.empty_like(L)
    out = torch.empty((2, 480, 640), dtype=torch.int16, device=dev)
    try:
        with _lib.use_context(ctx):
            for i in range(4):
                pair = [frames[i], frames[(i + 1) % 4]]
                L.copy_(torch.from_numpy(np.stack([q[0] for q in pair])))
                R.copy_(torch.from_numpy(np.stack([q[1] for q in pair])))
                b.compute(L, R, out)
                torch.cuda.synchronize()
                got = out.cpu().numpy()
                for k, (Lh, Rh) in enumerate(pair):
                    want = oracle.bm(Lh, Rh, bp)
                    assert np.array_equal(got[k], want), f"{cfg} call {i} frame {k}: " + report(got[k], want)
    finally:
        ctx.close()
