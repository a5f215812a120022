#!/usr/bin/env python
"""Diagnostic: the column-block carries the matrix-core wide Gram leaves in its workspace (linear seed, M = 2,
K(X), n = 5, L = 161: two column blocks), against numpy.  Prints the worst relative error per local pair."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from gpsig_amd import ops
    n, l, d, M = 5, 161, 46, 2
    rng = np.random.default_rng(3)
    X = np.cumsum(rng.standard_normal((n, l, d)), 1) / np.sqrt(l * d)
    Xt = torch.as_tensor(X, device="cuda", dtype=torch.float32)
    ops.sig_gram(Xt, None, M, base="linear")
    torch.cuda.synchronize()
    ws = ops.workspace(Xt.device, 1)
    q = (d + 3) // 4
    kq = q + ((2 - q % 4) + 4) % 4
    kp = 4 * kq
    rows = (l + 127 + 3) & ~3
    rec = 2 * rows * kp + 2 * rows
    off = (n * rec * 4 + 255) & ~255
    nrows, cw = l - 1, 4
    car = ws[off:off + 5 * 32 * nrows * cw * 4].view(torch.float32).cpu().numpy().reshape(5, 32, nrows, cw)
    dx = np.diff(X, axis=1)
    for b in range(n):
        for p in range(8):
            a = min(p, n - 1)
            c = dx[a] @ dx[b].T  # (nrows, ncell)
            exp = np.concatenate([np.zeros((1, 127)), np.cumsum(c[:, :127], 0)[:-1]], 0).sum(1)
            got = car[b, p, :, 0]
            print(b, p, float(np.abs(got - exp).max() / np.abs(exp).max()), got[:3], exp[:3])


if __name__ == "__main__":
    main()
