import sys, os, numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mvstereovision3_amd as mvsv
from oracle import pyoracle
SEED0 = 0x5EED0000
W, H = int(sys.argv[1]), int(sys.argv[2]); NF = int(sys.argv[3])
frames = [mvsv.synth_pair(SEED0 + i, W, H, 1, 128) for i in range(NF)]
Lt = torch.from_numpy(np.stack([f[0] for f in frames])).cuda()
Rt = torch.from_numpy(np.stack([f[1] for f in frames])).cuda()
for spk in (150, 0):
    m = mvsv.StereoSGBM.create(1, 128, 13, 0, 0, 0, 0, 0, spk, 2, mvsv.MODE_HH)
    a = m.compute(Lt, Rt).cpu().numpy()
    b = m.compute(Lt, Rt).cpu().numpy()
    p = {k: v for k, v in m.params().items() if k != "variant"}
    print("speckle", spk, "batch deterministic:", np.array_equal(a, b), "ndiff", int((a != b).sum()))
    for i in range(NF):
        single = m.compute(Lt[i], Rt[i]).cpu().numpy()
        want = pyoracle.sgbm(frames[i][0], frames[i][1], p)
        print(f"  frame {i}: batch==oracle {np.array_equal(a[i], want)} ({int((a[i]!=want).sum())})"
              f" single==oracle {np.array_equal(single, want)} ({int((single!=want).sum())})", flush=True)
