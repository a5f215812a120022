"""Isolate a wide-channel Gram mismatch: short x against long y at several channel counts / lengths."""
import sys, os
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpsig_amd import ops
from oracle import kernels_ref as kr


def walks(rng, n, L, D):
    return np.cumsum(rng.standard_normal((n, L, D)), 1) / np.sqrt(L * D)


for (D, L1, L2) in [(64, 3, 130), (64, 20, 130), (33, 3, 130), (64, 3, 100), (64, 3, 20), (9, 3, 130), (64, 9, 130), (64, 10, 130), (64, 130, 3), (64, 3, 300)]:
    rng = np.random.default_rng(D + L1 + L2)
    X, Y = walks(rng, 1, L1, D), walks(rng, 2, L2, D)
    for base in ("rbf", "linear"):
        ref = kr.SignatureKernelRef(L1 * D, D, 4, normalization=False, base=base).K_seq(X, Y)
        got = ops.sig_gram(torch.tensor(X, device="cuda"), torch.tensor(Y, device="cuda"), 4, base=base).double().cpu().numpy()
        err = [float(np.abs(got[m] - ref[m]).max() / max(np.abs(ref[m]).max(), 1e-30)) for m in range(1, 5)]
        print(D, L1, L2, base, ["%.1e" % e for e in err], flush=True)
