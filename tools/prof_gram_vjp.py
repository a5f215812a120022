"""Kernel-level profile driver for the Gram VJP (run under rocprofv3): N=1024, L=100, D=5, M=5,
K(X) upper-triangle pairs from the saved forward state.  Variants (three launches each, in order):
per-level upstream gradient; summed upstream gradient; summed + normalisation terms (rs, scale and
their gradients, as the autograd path of SignatureKernel.K passes them); per-level without state."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpsig_amd import ops  # noqa: E402

N, L, D, M = int(os.environ.get("N", 1024)), 100, 5, 5
rng = np.random.default_rng(0)
X = torch.tensor(np.cumsum(rng.standard_normal((N, L, D)), 1) / np.sqrt(L * D), device="cuda", dtype=torch.float32)
G = torch.randn(M + 1, N, N, device="cuda")
Gs = G.sum(0).contiguous()
rs = torch.rand(M + 1, N, device="cuda") + 0.5
sc = torch.rand(M + 1, device="cuda") + 0.5
grs = torch.zeros(M + 1, N, device="cuda")
gsc = torch.zeros(M + 1, device="cuda")
st = torch.empty(ops.sig_state_numel(N, None, L, M), dtype=torch.float32, device="cuda")
ops.sig_gram(X, None, M, state=st)
for _ in range(3):
    ops.sig_gram_vjp(X, None, M, G, gout_levels=True, state=st)
for _ in range(3):
    ops.sig_gram_vjp(X, None, M, Gs, state=st)
for _ in range(3):
    ops.sig_gram_vjp(X, None, M, Gs, state=st, rs1=rs, rs2=rs, scale=sc, jitter=1e-6, grs1=grs, grs2=grs,
                     gscale=gsc)
for _ in range(3):
    ops.sig_gram_vjp(X, None, M, G, gout_levels=True)
torch.cuda.synchronize()
