"""PCIe-inclusive rate of INTEGRATION.md 3a's tf.py_func binding at the headline shape (N=4096, L=128, D=5,
M=5): the py_func body (NumPy float64 sequences -> device fp32 -> raw levels -> float64 NumPy on the host)
against the same Gram with the inputs and output resident on the device.  One JSON line.

  python tools/bench_pcie.py [--n 4096] [--reps 5]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpsig_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--l", type=int, default=128)
    ap.add_argument("--d", type=int, default=5)
    ap.add_argument("--m", type=int, default=5)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    rng = np.random.default_rng(0)
    x = np.cumsum(rng.standard_normal((a.n, a.l, a.d)), 1) / np.sqrt(a.l * a.d)
    dev = torch.device("cuda")

    def host_call(xn):  # the py_func body of INTEGRATION.md 3a
        xs = torch.from_numpy(np.ascontiguousarray(xn)).to(dev, torch.float32)
        return ops.sig_gram(xs, None, a.m).double().cpu().numpy()

    xd = torch.tensor(x, device=dev, dtype=torch.float32)
    host_call(x)
    ops.sig_gram(xd, None, a.m)
    torch.cuda.synchronize()
    th = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        host_call(x)
        th.append(time.perf_counter() - t0)
    td = []
    for _ in range(a.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ops.sig_gram(xd, None, a.m)
        torch.cuda.synchronize()
        td.append(time.perf_counter() - t0)
    th, td = float(np.median(th)), float(np.median(td))
    entries = a.n * a.n
    print(json.dumps({"workload": f"K(X) raw levels N={a.n} L={a.l} D={a.d} M={a.m}", "reps": a.reps,
                      "host_roundtrip_ms": th * 1e3, "device_resident_ms": td * 1e3,
                      "pcie_inclusive_entries_per_s": entries / th, "device_entries_per_s": entries / td,
                      "bytes_h2d": x.size * 8, "bytes_d2h": (a.m + 1) * entries * 8}))


if __name__ == "__main__":
    main()
