"""Failure surfacing and stream ordering of the HIP path (through the C ABI).

* A strip-to-strip hand-off of the sheared-strip SGBM kernel that gives up
  (forced with MVSV_OPT_STRIP_SPIN_LIMIT = 0) must never yield a computed map:
  the launch's maps come back all INVALID, the error surfaces as
  MvsvError(MVSV_E_TIMEOUT) on the device path (next call / synchronize), the
  host path and the frame stream, and the next call is bit-exact again.
* Device calls on torch's stream followed at once by a host call on the
  context's own stream (no synchronisation in between) share the context's
  buffers: the stream switch must order them.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED0 = 0x5EED0000


def sgbm_yml_matcher(mvsv, mode=1):
    import os
    m = mvsv.StereoSGBM.create(0, 0, 0, 0, 0)
    para = mvsv.sgbmParameters()
    here = os.path.dirname(os.path.abspath(__file__))
    assert mvsv.Disparity.loadSGBMParameters(os.path.join(here, "golden", "configs", "sgbm.yml"),
                                             m, para)
    m.setMode(mode)
    return m


def oracle_params(m):
    p = dict(m.params())
    p.pop("variant")
    return p


@pytest.fixture
def restore_spin_limit(mvsv):
    # the sheared-strip schedule (small launches would run the line directions
    # side by side, which have no hand-off to give up)
    mvsv.set_option(mvsv.OPT_PATH_SCHEDULE, 1)
    yield
    mvsv.set_option(mvsv.OPT_PATH_SCHEDULE, 0)
    mvsv.set_option(mvsv.OPT_STRIP_SPIN_LIMIT, 1 << 20)
    try:
        mvsv.synchronize()
    except mvsv.MvsvError:
        pass


def test_strip_timeout_device_path(gpu, mvsv, oracle, restore_spin_limit):
    import torch
    W, H, F = 640, 480, 4
    m = sgbm_yml_matcher(mvsv)
    pairs = [mvsv.synth_pair(SEED0 + 900 + i, W, H, 1, 128) for i in range(F)]
    Lt = torch.from_numpy(np.stack([p[0] for p in pairs])).cuda()
    Rt = torch.from_numpy(np.stack([p[1] for p in pairs])).cuda()
    mvsv.synchronize()
    mvsv.set_option(mvsv.OPT_STRIP_SPIN_LIMIT, 0)  # give up at the first not-ready poll
    out = m.compute(Lt, Rt)
    with pytest.raises(mvsv.MvsvError) as ei:
        mvsv.synchronize()
    assert ei.value.code == mvsv.MVSV_E_TIMEOUT
    invalid = (m.getMinDisparity() - 1) * 16
    assert bool((out == invalid).all()), "a map computed after a given-up wait left the pipeline"
    # the error is reported once; the next call on the same context is exact again
    mvsv.set_option(mvsv.OPT_STRIP_SPIN_LIMIT, 1 << 20)
    out2 = m.compute(Lt, Rt)
    mvsv.synchronize()
    want = oracle.sgbm(pairs[0][0], pairs[0][1], oracle_params(m))
    assert np.array_equal(out2[0].cpu().numpy(), want)


def test_strip_timeout_reported_by_next_device_call(gpu, mvsv, oracle, restore_spin_limit):
    import torch
    W, H = 640, 480
    m = sgbm_yml_matcher(mvsv)
    L, R = mvsv.synth_pair(SEED0 + 910, W, H, 1, 128)
    Lt = torch.from_numpy(np.stack([L] * 4)).cuda()
    Rt = torch.from_numpy(np.stack([R] * 4)).cuda()
    mvsv.synchronize()
    mvsv.set_option(mvsv.OPT_STRIP_SPIN_LIMIT, 0)
    m.compute(Lt, Rt)
    torch.cuda.synchronize()  # the launch has completed; no mvsv check yet
    mvsv.set_option(mvsv.OPT_STRIP_SPIN_LIMIT, 1 << 20)
    with pytest.raises(mvsv.MvsvError) as ei:
        m.compute(Lt, Rt)  # reports the earlier launch's give-up before enqueueing
    assert ei.value.code == mvsv.MVSV_E_TIMEOUT
    got = m.compute(Lt[:1], Rt[:1])
    mvsv.synchronize()
    assert np.array_equal(got[0].cpu().numpy(), oracle.sgbm(L, R, oracle_params(m)))


def test_strip_timeout_host_path(gpu, mvsv, oracle, restore_spin_limit):
    m = sgbm_yml_matcher(mvsv)
    L, R = mvsv.synth_pair(SEED0 + 920, 1280, 960, 1, 128)
    mvsv.set_option(mvsv.OPT_STRIP_SPIN_LIMIT, 0)
    with pytest.raises(mvsv.MvsvError) as ei:
        m.compute(L, R)
    assert ei.value.code == mvsv.MVSV_E_TIMEOUT
    mvsv.set_option(mvsv.OPT_STRIP_SPIN_LIMIT, 1 << 20)
    got = m.compute(L, R)
    assert np.array_equal(got, oracle.sgbm(L, R, oracle_params(m)))


def test_strip_timeout_stream_frames(gpu, mvsv, oracle, restore_spin_limit):
    W, H = 640, 480
    m = sgbm_yml_matcher(mvsv)
    frames = [mvsv.synth_pair(SEED0 + 930 + i, W, H, 1, 128) for i in range(4)]
    mvsv.set_option(mvsv.OPT_STRIP_SPIN_LIMIT, 0)
    st = mvsv.DisparityStream(m, W, H, depth=4, batch=2)
    st.push(*frames[0])
    st.push(*frames[1])  # a full group: launched with the zero limit
    import torch
    torch.cuda.synchronize()
    mvsv.set_option(mvsv.OPT_STRIP_SPIN_LIMIT, 1 << 20)
    st.push(*frames[2])
    st.push(*frames[3])
    for _ in range(2):  # both frames of the failed launch report it
        with pytest.raises(mvsv.MvsvError) as ei:
            st.pop()
        assert ei.value.code == mvsv.MVSV_E_TIMEOUT
    for i in (2, 3):
        d, _ = st.pop()
        assert np.array_equal(d, oracle.sgbm(*frames[i], oracle_params(m))), f"frame {i}"
    st.close()


def test_stream_switch_orders_shared_buffers(gpu, mvsv, oracle):
    """compute(torch) then compute(numpy) with no sync: the host call runs on the
    context's own stream and must wait for the device call that shares its buffers."""
    import torch
    m = sgbm_yml_matcher(mvsv)
    a = mvsv.synth_pair(SEED0 + 940, 1280, 960, 1, 128)
    b = mvsv.synth_pair(SEED0 + 941, 1280, 960, 1, 128)
    Lt = torch.from_numpy(np.stack([a[0]] * 8)).cuda()
    Rt = torch.from_numpy(np.stack([a[1]] * 8)).cuda()
    torch.cuda.synchronize()
    dev_out = m.compute(Lt, Rt)  # 8-frame launch on torch's stream, not waited for
    host_out = m.compute(b[0], b[1])  # host path, context stream
    torch.cuda.synchronize()
    p = oracle_params(m)
    assert np.array_equal(host_out, oracle.sgbm(b[0], b[1], p))
    want_a = oracle.sgbm(a[0], a[1], p)
    got = dev_out.cpu().numpy()
    for f in range(8):
        assert np.array_equal(got[f], want_a), f"device frame {f}"


def test_entry_points_restore_current_device(gpu, mvsv):
    import torch
    m = mvsv.StereoSGBM.create(0, 32, 5)
    L, R = mvsv.synth_pair(SEED0 + 950, 160, 64, 0, 32)
    torch.cuda.set_device(0)
    before = torch.cuda.current_device()
    m.compute(L, R)
    m.compute(torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda())
    mvsv.synchronize()
    assert torch.cuda.current_device() == before


def test_stream_switch_after_caller_stream_destroyed(gpu, mvsv, oracle):
    """A device call on a caller-owned HIP stream, the caller destroys that
    stream, then a host call switches the context to its own stream: the switch
    waits on the context's own last-use event and never touches the destroyed
    handle (recording on it was undefined behaviour)."""
    import ctypes
    import torch
    hip = ctypes.CDLL("libamdhip64.so")
    h = ctypes.c_void_p()
    assert hip.hipStreamCreate(ctypes.byref(h)) == 0
    m = sgbm_yml_matcher(mvsv)
    a = mvsv.synth_pair(SEED0 + 960, 320, 240, 1, 128)
    b = mvsv.synth_pair(SEED0 + 961, 320, 240, 1, 128)
    Lt = torch.from_numpy(a[0]).cuda()
    Rt = torch.from_numpy(a[1]).cuda()
    ext = torch.cuda.ExternalStream(h.value)
    with torch.cuda.stream(ext):
        dev_out = m.compute(Lt, Rt)
    ext.synchronize()
    got_a = dev_out.cpu().numpy()
    del ext
    assert hip.hipStreamDestroy(h) == 0
    host_out = m.compute(b[0], b[1])  # switches to the context's own stream
    p = oracle_params(m)
    assert np.array_equal(got_a, oracle.sgbm(a[0], a[1], p))
    assert np.array_equal(host_out, oracle.sgbm(b[0], b[1], p))
    mvsv.synchronize()
