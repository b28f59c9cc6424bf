"""Batches in flight (mvstereovision3_amd.batch.InflightBatches, bench.py
--inflight): consecutive steps on separate HIP streams and contexts overlap on
the GPU; every slot's maps stay bit-exact against the oracle, and a slot's
context never sees another slot's launches (use_context)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_inflight_batches_bit_exact(gpu, mvsv, oracle):
    torch = gpu
    from mvstereovision3_amd import _lib
    from mvstereovision3_amd.batch import InflightBatches
    W, H, F = 320, 240, 2
    m = mvsv.StereoSGBM.create(1, 128, 13, 0, 0, 0, 0, 0, 150, 2, 1)
    pairs = [mvsv.synth_pair(0x5EED0000 + 500 + i, W, H, 1, 128) for i in range(F)]
    dev = torch.device("cuda", 0)
    Lt = torch.from_numpy(np.stack([p[0] for p in pairs])).to(dev)
    Rt = torch.from_numpy(np.stack([p[1] for p in pairs])).to(dev)
    b = InflightBatches(Lt, Rt, lambda: torch.full((F, H, W), -7, dtype=torch.int16, device=dev),
                        lambda L, R, o: m.compute(L, R, o), 3, dev)
    for _ in range(7):
        b.step()
    b.join()
    torch.cuda.synchronize()
    for c in b.contexts():
        _lib.check(_lib.lib().mvsv_synchronize(c.handle), c.handle)
    p = {k: v for k, v in m.params().items() if k != "variant"}
    want = [oracle.sgbm(L, R, p) for L, R in pairs]
    for _, _, out in b.slots:
        got = out.cpu().numpy()
        for f in range(F):
            assert np.array_equal(got[f], want[f])
    # the thread's default context is untouched by the slots
    assert _lib.context(0) not in b.contexts()
