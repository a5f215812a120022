"""Precision of the split-f16 matrix-core wide Gram (sig_fo_mf.h) against the fp64 oracle, per level
(norm-relative), next to the fp32 channel-loop kernel (GPSIG_WIDE_MF=0 in a child process) on the same inputs.

    python tools/diag_mf_precision.py [--mf 0|1]   (prints one JSON line per shape)
"""
import argparse
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SHAPES = [(33, 64), (46, 136), (63, 128), (126, 128), (126, 136), (46, 500), (200, 100), (16, 128), (9, 100)]


def walks(rng, n, l, d, s=1.0):
    return (np.cumsum(rng.standard_normal((n, l, d)), 1) * s / np.sqrt(l * d))


def run():
    import torch
    from gpsig_amd import ops
    from oracle import kernels_ref as kr
    out = []
    for d, l in SHAPES:
        rng = np.random.default_rng(d * 1000 + l)
        M = 4
        X = walks(rng, 6, l, d)
        ref = kr.SignatureKernelRef(l * d, d, M, normalization=False).K_seq(X)
        got = ops.sig_gram(torch.tensor(X, dtype=torch.float32, device="cuda"), None, M).cpu().numpy().astype(np.float64)
        err = [float(np.linalg.norm(got[m] - ref[m]) / np.linalg.norm(ref[m])) for m in range(1, M + 1)]
        out.append(dict(d=d, l=l, mf=os.environ.get("GPSIG_WIDE_MF", "1"), level_err=err,
                        max_abs=float(np.abs(got - ref).max()), max_ref=float(np.abs(ref).max())))
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--child", action="store_true")
    a = ap.parse_args()
    if a.child:
        for o in run():
            print(json.dumps(o), flush=True)
    else:
        for mf in ("1", "0"):
            r = subprocess.run([sys.executable, __file__, "--child"], env=dict(os.environ, GPSIG_WIDE_MF=mf),
                               capture_output=True, text=True, timeout=600)
            sys.stdout.write(r.stdout)
            if r.returncode:
                sys.stderr.write(r.stderr[-3000:])
                sys.exit(r.returncode)
