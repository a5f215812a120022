"""Kernel-level profile driver for the Gram VJP (run under rocprofv3): N=1024, L=100, D=5, M=5,
K(X) upper-triangle pairs; three VJP launches from the saved forward state, three recomputing it."""
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
st = torch.empty(ops.sig_state_numel(N, None, L, M), dtype=torch.float32, device="cuda")
ops.sig_gram(X, None, M, state=st)
for use_state in (True, False):
    for _ in range(3):
        ops.sig_gram_vjp(X, None, M, G, gout_levels=True, state=st if use_state else None)
torch.cuda.synchronize()
