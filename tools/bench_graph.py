#!/usr/bin/env python
"""Eager vs hipGraph-replayed K(X) on small problems (launch-bound): median wall time per call,
device-synchronised.  One JSON object per line.

    python tools/bench_graph.py
"""
import json
import os
import statistics
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gpsig_amd  # noqa: E402
from gpsig_amd.graphs import GraphedCall  # noqa: E402


def timed(fn, reps=50):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts) * 1e3


def main():
    for (n, l, d, m) in [(64, 50, 3, 4), (256, 50, 3, 4), (1024, 100, 5, 5)]:
        rng = np.random.default_rng(0)
        X = torch.tensor(np.cumsum(rng.standard_normal((n, l, d)), 1).reshape(n, -1) / np.sqrt(l * d),
                         device="cuda", dtype=torch.float32)
        k = gpsig_amd.SignatureRBF(l * d, d, m).to("cuda")
        g = GraphedCall(lambda a: k.K(a), X)
        with torch.no_grad():
            te = timed(lambda: k.K(X))
        tg = timed(lambda: g(X))
        print(json.dumps({"workload": f"SignatureRBF K(X) normalised N={n} L={l} D={d} M={m}",
                          "eager_ms": te, "graph_ms": tg, "speedup": te / tg}), flush=True)


if __name__ == "__main__":
    main()
