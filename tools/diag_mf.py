#!/usr/bin/env python
"""Diagnostic: raw per-level Grams of the wide first-order path on one case, saved for an A/B between the
matrix-core kernel (default) and the runtime channel loop (GPSIG_WIDE_MF=0, set by the caller).

    python tools/diag_mf.py OUT.npz --n 5 --l 300 --l2 293 --d 46 --m 4 [--sym]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--n", type=int, default=5)
    ap.add_argument("--n2", type=int, default=3)
    ap.add_argument("--l", type=int, default=300)
    ap.add_argument("--l2", type=int, default=0)
    ap.add_argument("--d", type=int, default=46)
    ap.add_argument("--m", type=int, default=4)
    ap.add_argument("--base", default="rbf")
    a = ap.parse_args()
    import torch
    from gpsig_amd import ops
    rng = np.random.default_rng(a.d * 1000 + a.l)
    X = np.cumsum(rng.standard_normal((a.n, a.l, a.d)), 1) / np.sqrt(a.l * a.d)
    Y = np.cumsum(rng.standard_normal((a.n2, a.l2 or a.l, a.d)), 1) / np.sqrt(a.l * a.d)
    t = lambda v: torch.as_tensor(v, device="cuda")
    rect = ops.sig_gram(t(X), t(Y), a.m, base=a.base).cpu().numpy()
    sym = ops.sig_gram(t(X), None, a.m, base=a.base).cpu().numpy()
    np.savez(a.out, rect=rect, sym=sym)


if __name__ == "__main__":
    main()
