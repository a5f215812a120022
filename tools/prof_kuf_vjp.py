"""Profile driver for the tens-vs-seq VJP (run under rocprofv3): T=512 tensors x N=1024 sequences,
L=100, D=5, M=5, RBF difference seed, increments False; three VJP launches."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpsig_amd import ops  # noqa: E402

T, N, L, D, M = 512, 1024, 100, 5, 5
rng = np.random.default_rng(0)
X = torch.tensor(np.cumsum(rng.standard_normal((N, L, D)), 1) / np.sqrt(L * D), device="cuda", dtype=torch.float32)
Z = torch.tensor(rng.standard_normal((M * (M + 1) // 2, T, D)), device="cuda", dtype=torch.float32)
G = torch.randn(M + 1, T, N, device="cuda")
for _ in range(3):
    ops.tens_vs_seq_vjp(Z, X, M, G)
torch.cuda.synchronize()
