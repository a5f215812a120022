"""Raw-level higher-order Gram VJP timings (ops.sig_gram_vjp, gout per level) for the one-wave LDS-state kernel
(l2 <= 256) and the split kernel (257-509 points).  One JSON line per case; inputs resident, median of reps.

    python tools/bench_ho_vjp.py [--reps 5]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpsig_amd import ops  # noqa: E402

CASES = [  # (N, L, D, M, order, base): symmetric K(X) VJP over the upper triangle
    (64, 100, 5, 4, 4, "rbf"),
    (64, 200, 5, 5, 5, "linear"),
    (64, 150, 5, 6, 3, "rbf"),
    (32, 256, 4, 5, 5, "rbf"),
    (16, 500, 24, 5, 5, "linear"),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda")
    for n, l, d, m, o, base in CASES:
        X = torch.tensor(np.cumsum(np.random.default_rng(0).standard_normal((n, l, d)), 1) / np.sqrt(l * d),
                         device=dev, dtype=torch.float32)
        G = torch.randn((m + 1, n, n), device=dev)
        f = lambda: ops.sig_gram_vjp(X, None, m, G, base=base, gout_levels=True, order=o)
        f()
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            f()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        print(json.dumps({"N": n, "L": l, "D": d, "M": m, "order": o, "base": base, "ms": float(np.median(ts))}),
              flush=True)


if __name__ == "__main__":
    main()
