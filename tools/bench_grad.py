#!/usr/bin/env python
"""Forward and forward+backward time of the normalised K(X) (SignatureRBF, order 1) on one GPU, and the
gradient's error vs torch fp64 autodiff of the reference graph (oracle/autodiff_ref.py) on a subsample.

    python tools/bench_grad.py --n 1024 --l 100 --d 5 --m 5
"""
import argparse
import json
import os
import statistics
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--l", type=int, default=100)
    ap.add_argument("--d", type=int, default=5)
    ap.add_argument("--m", type=int, default=5)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--check", type=int, default=8, help="sequences in the fp64 autodiff check (0 = skip)")
    a = ap.parse_args()
    import gpsig_amd
    from oracle import autodiff_ref as ar
    rng = np.random.default_rng(0)
    Xnp = np.cumsum(rng.standard_normal((a.n, a.l, a.d)), axis=1) / np.sqrt(a.l * a.d)
    X = torch.tensor(Xnp.reshape(a.n, -1), device="cuda", dtype=torch.float32)
    G = torch.randn(a.n, a.n, device="cuda")
    k = gpsig_amd.SignatureRBF(a.l * a.d, a.d, a.m)

    def fwd():
        with torch.no_grad():
            return k.K(X)

    def fwdbwd():
        Xg = X.detach().requires_grad_(True)
        (k.K(Xg) * G).sum().backward()
        return Xg.grad

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        return statistics.median(ts)

    tf, tb = timed(fwd), timed(fwdbwd)
    res = dict(workload=f"SignatureRBF K(X) normalised N={a.n} L={a.l} D={a.d} M={a.m}", fwd_ms=tf * 1e3,
               fwd_bwd_ms=tb * 1e3, bwd_over_fwd=(tb - tf) / tf, entries_per_s_fwd_bwd=a.n * a.n / tb)
    if a.check:
        S = a.check
        Xs = torch.tensor(Xnp[:S].reshape(S, -1), device="cuda", requires_grad=True)
        Gs = torch.randn(S, S, dtype=torch.float64)
        (k.K(Xs) * Gs.to("cuda")).sum().backward()
        Xr = torch.tensor(Xnp[:S], requires_grad=True)
        (ar.K(Xr, None, a.m) * Gs).sum().backward()
        g, r = Xs.grad.reshape(Xr.shape).cpu().numpy(), Xr.grad.numpy()
        res["grad_norm_rel_err"] = float(np.abs(g - r).max() / np.abs(r).max())
    print(json.dumps(res))


if __name__ == "__main__":
    main()
