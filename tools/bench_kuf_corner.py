"""Kuf forward (ops.tens_vs_seq, increments=True, RBF) at the SVGP shapes (T = 500 inducing tensors, N = 50
sequences of 500 points, D = 126, num_levels = 4) in two regimes: the benchmark's small increments (the
chained expm1 recurrences) and increments far apart (|q| or |c| >= 2 on about half the steps: the corner
differences of directly evaluated base-kernel values).  One JSON line per regime: ms per call."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpsig_amd import ops  # noqa: E402


def main(reps=10, t=500, n=50, l=500, d=126, m=4):
    lt = m * (m + 1) // 2
    rng = np.random.default_rng(3)
    Z = torch.tensor(rng.standard_normal((lt, t, 2, d)) / np.sqrt(d), device="cuda", dtype=torch.float32)
    for regime, scale in (("small_increments", 1.0 / np.sqrt(l * d)), ("corner", 1.5 / np.sqrt(d))):
        X = torch.tensor(np.cumsum(rng.standard_normal((n, l, d)) * scale, 1), device="cuda", dtype=torch.float32)
        ops.tens_vs_seq(Z, X, m, increments=True)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            out = ops.tens_vs_seq(Z, X, m, increments=True)
        e1.record()
        torch.cuda.synchronize()
        print(json.dumps(dict(regime=regime, workload=f"Kuf T={t} N={n} L={l} D={d} M={m} increments",
                              ms=e0.elapsed_time(e1) / reps, finite=bool(torch.isfinite(out).all()))), flush=True)


if __name__ == "__main__":
    main()
