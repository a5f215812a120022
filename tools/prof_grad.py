"""Kernel-level profile driver for the backward paths (run under rocprofv3 --kernel-trace --stats):
PDE Kdiag fwd+bwd (N=1024, L=200, D=5, dyadic 1) and Gram K(X) fwd+bwd (N=512, L=100, D=5, M=5)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gpsig_amd  # noqa: E402

rng = np.random.default_rng(0)
X = torch.tensor(np.cumsum(rng.standard_normal((1024, 200, 5)), 1).reshape(1024, -1) / np.sqrt(1000),
                 device="cuda", dtype=torch.float32)
kp = gpsig_amd.UntruncSignatureKernel(1000, 5, order=1)
w = torch.randn(1024, device="cuda")
X2 = torch.tensor(np.cumsum(rng.standard_normal((512, 100, 5)), 1).reshape(512, -1) / np.sqrt(500),
                  device="cuda", dtype=torch.float32)
k = gpsig_amd.SignatureRBF(500, 5, 5)
G = torch.randn(512, 512, device="cuda")
for _ in range(3):
    Xg = X.detach().requires_grad_(True)
    (kp.Kdiag(Xg) * w).sum().backward()
    X2g = X2.detach().requires_grad_(True)
    (k.K(X2g) * G).sum().backward()
torch.cuda.synchronize()
