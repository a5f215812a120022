#!/usr/bin/env python
"""Wide-channel rows: raw K(X) Gram launch time (HIP events, median) of the first-order RBF kernel at
channel counts the reference's runners feed, and the A/B of the wide kernels (runtime channel loop,
wide.h) against the fixed instantiations where both exist (GPSIG_FO_FIXED_MAX=0 forces wide).

    python tools/bench_wide.py [--n 1024] [--l 128] [--m 4] [--d 8 16 32 46 126] > rows.jsonl
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--l", type=int, default=128)
    ap.add_argument("--m", type=int, default=4)
    ap.add_argument("--d", type=int, nargs="+", default=[8, 16, 32, 46, 126])
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import torch
    from gpsig_amd import ops
    dev = torch.device("cuda", 0)
    for d in args.d:
        rng = np.random.default_rng(d)
        X = torch.as_tensor(np.cumsum(rng.standard_normal((args.n, args.l, d)), 1) / np.sqrt(args.l * d),
                            device=dev, dtype=torch.float32)
        for _ in range(2):
            ops.sig_gram(X, None, args.m)
        torch.cuda.synchronize()
        ts = []
        for _ in range(args.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            ops.sig_gram(X, None, args.m)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        ms = statistics.median(ts)
        pairs = args.n * (args.n + 1) // 2
        cells = pairs * (args.l - 1) ** 2
        B = 4 * (args.l - 1) ** 2 + 4 * (args.m + 1)
        print(json.dumps({"n": args.n, "l": args.l, "d": d, "m": args.m,
                          "fixed_max": os.environ.get("GPSIG_FO_FIXED_MAX", "8"), "ms": round(ms, 3),
                          "cells_per_s": cells / (ms * 1e-3), "frac_8d": pairs * B / (ms * 1e-3) / 8e12,
                          "dot_tflops": cells * 1.25 * d * 2 / (ms * 1e-3) / 1e12}), flush=True)


if __name__ == "__main__":
    main()
