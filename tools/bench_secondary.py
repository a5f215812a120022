#!/usr/bin/env python
"""Timing of the secondary paths (not BASELINE rows): linear and higher-order Grams, PDE at other
dyadic orders, the tensor Gram.  Median of 5 device-synchronised calls, inputs resident."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpsig_amd import ops  # noqa: E402


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return sorted(ts)[len(ts) // 2] * 1e3


rng = np.random.default_rng(0)


def walks(n, l, d):
    return torch.tensor(np.cumsum(rng.standard_normal((n, l, d)), 1) / np.sqrt(l * d), device="cuda",
                        dtype=torch.float32)


X = walks(1024, 100, 5)
res = {}
res["gram_rbf_o1_N1024_L100_M5_ms"] = timed(lambda: ops.sig_gram(X, None, 5))
res["gram_lin_o1_N1024_L100_M5_ms"] = timed(lambda: ops.sig_gram(X, None, 5, base="linear"))
res["gram_rbf_o2_N1024_L100_M5_ms"] = timed(lambda: ops.sig_gram(X, None, 5, order=2))
Xs = walks(256, 64, 4)
res["gram_lin_oM_N256_L64_M5_ms"] = timed(lambda: ops.sig_gram(Xs, None, 5, order=5, base="linear"))
# the exact signature kernel at the reference's VOSF training shape (max_len 500 is the data's; L=100 here):
# signature features + per-level GEMMs vs the higher-order recursion (order = num_levels - 1 forces it)
Xv = walks(1024, 100, 5)
res["gram_lin_oM_N1024_L100_D5_M4_features_ms"] = timed(lambda: ops.sig_gram(Xv, None, 4, order=4, base="linear"))
ops_max = ops.SIG_FEATURE_MAX
ops.SIG_FEATURE_MAX = 0
res["gram_lin_oM_N1024_L100_D5_M4_recursion_ms"] = timed(lambda: ops.sig_gram(Xv, None, 4, order=4, base="linear"))
ops.SIG_FEATURE_MAX = ops_max
Xp = walks(512, 100, 5)
for dy in (0, 2):
    res[f"pde_gram_N512_L100_dyadic{dy}_ms"] = timed(lambda: ops.pde_gram(Xp, None, dy, 1))
Z = torch.tensor(rng.standard_normal((15, 512, 5)), device="cuda", dtype=torch.float32)
res["tens_gram_T512_M5_ms"] = timed(lambda: ops.tens_gram(Z, 5))
print(json.dumps(res))
