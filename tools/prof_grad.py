"""Kernel-level profile driver for the backward paths (run under rocprofv3 --kernel-trace --stats), three
training steps each: PDE Kdiag fwd+bwd (N=1024, L=200, D=5, dyadic 1), PDE cross Gram fwd+bwd (256 x 256,
L=100, dyadic 1), Gram K(X) fwd+bwd (N=512, L=100, D=5, M=5), Kuf fwd+bwd (T=512 x N=1024, L=100, M=5)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gpsig_amd  # noqa: E402

rng = np.random.default_rng(0)


def walks(n, l, d):
    return torch.tensor(np.cumsum(rng.standard_normal((n, l, d)), 1).reshape(n, -1) / np.sqrt(l * d),
                        device="cuda", dtype=torch.float32)


X = walks(1024, 200, 5)
kp = gpsig_amd.UntruncSignatureKernel(1000, 5, order=1)
w = torch.randn(1024, device="cuda")
Xa, Xb = walks(256, 100, 5), walks(256, 100, 5)
kq = gpsig_amd.UntruncSignatureKernel(500, 5, order=1)
Gq = torch.randn(256, 256, device="cuda")
X2 = walks(512, 100, 5)
k = gpsig_amd.SignatureRBF(500, 5, 5)
G = torch.randn(512, 512, device="cuda")
X3 = walks(1024, 100, 5)
Z = torch.tensor(rng.standard_normal((15, 512, 5)), device="cuda", dtype=torch.float32)
Gz = torch.randn(512, 1024, device="cuda")
for _ in range(3):
    Xg = X.detach().requires_grad_(True)
    (kp.Kdiag(Xg) * w).sum().backward()
    Xag = Xa.detach().requires_grad_(True)
    (kq.K(Xag, Xb) * Gq).sum().backward()
    X2g = X2.detach().requires_grad_(True)
    (k.K(X2g) * G).sum().backward()
    Zg, X3g = Z.detach().requires_grad_(True), X3.detach().requires_grad_(True)
    (k.K_tens_vs_seq(Zg, X3g) * Gz).sum().backward()
torch.cuda.synchronize()
