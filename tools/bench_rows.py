#!/usr/bin/env python
"""Measure the SURVEY.md §8 configurations other than the headline (bench.py measures H):

  C2  SignatureRBF K(X) normalised, N=1024, L=100, D=5, M=5
  C3  PDE signature-kernel Gram K(X), N=1024, L=200, D=5, dyadic=1, solver=1
  C4  inducing-tensor Kuf (K_tens_vs_seq, normalised), T=512 x N=4096, L=100, M=5, increments False/True
  C5  SignatureRBF K(X) normalised, N=8192, L=128, D=8, M=6 on ONE GPU (the 8-GPU config's work)
  W46, W126  SignatureRBF K(X) normalised at the reference runners' wide channel counts (VERDICT r2 #1:
      (D+1)*2 = 46 AUSLAN, 126 CMU/KickvsPunch/WalkvsRun): N=1024, L=136 / 128, M=4 (runtime channel loop)
  P128  PDE Gram K(X) at d = 128 (the VOSF-RNN's num_hidden, train_gpsigrnn_vosf.py:74,82): N=256, L=100,
      dyadic 1 (increment-tile mode: GEMM of the increments, then the solver)

Per config: whole-call entries/s (median of --reps device-synchronised runs, inputs resident), the
dominant kernel's launch time from HIP events on its stream, the §8d effective-bandwidth roofline,
max-abs error vs the fp64 oracle on a subsample, and a bounded CPU-baseline sample (oracle, host
cores).  Writes one JSON object per config to stdout (and --out).

    python tools/bench_rows.py --out profiles/r1_rows.json
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
HBM_PEAK_GBS = 8000.0


def walks(n, l, d, seed):
    rng = np.random.default_rng(seed)
    return (np.cumsum(rng.standard_normal((n, l, d)), axis=1) / np.sqrt(l * d)).astype(np.float32)


def timed(fn, reps, warm=2):
    import torch
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts)


def kernel_ms(fn):
    """Events bracketing one call on the current stream (the library launches on it)."""
    import torch
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1)


def cpu_rate(fn, units, seconds):
    t0 = time.perf_counter()
    done = 0
    while time.perf_counter() - t0 < seconds:
        fn()
        done += units
    return done / (time.perf_counter() - t0)


def row_gram(name, n, l, d, m, reps, cpu_s):
    import torch
    import gpsig_amd
    from gpsig_amd import ops
    from oracle import kernels_ref as kr
    dev = torch.device("cuda", 0)
    Xnp = walks(n, l, d, 0)
    X = torch.as_tensor(Xnp.reshape(n, -1), device=dev)
    k = gpsig_amd.SignatureRBF(l * d, d, m)
    t = timed(lambda: k.K(X), reps)
    Xs = k._prep(X)
    kms = kernel_ms(lambda: ops.sig_gram(Xs, None, m))
    K = k.K(X)
    S = np.unique(np.linspace(0, n - 1, 48).astype(int))
    ref = kr.SignatureKernelRef(l * d, d, m).K(Xnp[S].astype(np.float64).reshape(len(S), -1))
    got = K[torch.as_tensor(S, device=dev)][:, torch.as_tensor(S, device=dev)].double().cpu().numpy()
    b_entry = 4 * (l - 1) ** 2 + 4 * (m + 1)
    kn = kr.SignatureKernelRef(l * d, d, m, normalization=False)
    Xc = Xnp[:16].astype(np.float64)
    cpu = cpu_rate(lambda: kn.K_seq(Xc[:4], Xc[4:8]), 16, cpu_s)
    return dict(config=name, workload=f"SignatureRBF K(X) normalised N={n} L={l} D={d} M={m}",
                entries_per_s=n * n / t, ms_per_call=t * 1e3, gram_kernel_ms=kms,
                # the symmetric launch evaluates the n(n+1)/2 pairs b >= a (the mirror is a store)
                roofline=dict(bytes_per_entry=b_entry, pairs_per_launch=n * (n + 1) // 2,
                              achieved_GBs=n * (n + 1) / 2 * b_entry / (kms / 1e3) / 1e9,
                              frac=n * (n + 1) / 2 * b_entry / (kms / 1e3) / 1e9 / HBM_PEAK_GBS),
                max_abs_err=float(np.abs(got - ref).max()),
                cpu_baseline=dict(entries_per_s=cpu, cores=1, kind="port",
                                  sample="4x4-pair raw Gram blocks, oracle/kernels_ref.py fp64 NumPy, 1 process"))


def row_pde(reps, cpu_s, n=1024, l=200, d=5, dy=1, name="C3"):
    import torch
    from gpsig_amd import ops
    from oracle import pde
    dev = torch.device("cuda", 0)
    Xnp = walks(n, l, d, 0)
    X = torch.as_tensor(Xnp, device=dev)
    t = timed(lambda: ops.pde_gram(X, None, dy, 1), reps)
    kms = kernel_ms(lambda: ops.pde_gram(X, None, dy, 1))
    K = ops.pde_gram(X, None, dy, 1)
    S = np.unique(np.linspace(0, n - 1, 24).astype(int))
    ref = pde.pde_gram(Xnp[S].astype(np.float64), None, dy, 1)
    got = K[torch.as_tensor(S, device=dev)][:, torch.as_tensor(S, device=dev)].double().cpu().numpy()
    b_entry = 4 * (l - 1) ** 2 + 4
    threads = min(len(os.sched_getaffinity(0)), int(os.environ.get("OMP_NUM_THREADS", "16")))
    Xc = Xnp[:16].astype(np.float64)
    cpu = cpu_rate(lambda: pde.pde_gram(Xc[:8], Xc[8:16], dy, 1), 64, cpu_s)
    return dict(config=name, workload=f"PDE Gram K(X) N={n} L={l} D={d} dyadic={dy} solver=1 (fp64 solution)",
                entries_per_s=n * n / t, ms_per_call=t * 1e3, pde_kernel_ms=kms,
                roofline=dict(bytes_per_entry=b_entry, pairs_per_launch=n * (n + 1) // 2,
                              achieved_GBs=n * (n + 1) / 2 * b_entry / (kms / 1e3) / 1e9,
                              frac=n * (n + 1) / 2 * b_entry / (kms / 1e3) / 1e9 / HBM_PEAK_GBS),
                max_abs_err=float(np.abs(got - ref).max()), max_abs_ref=float(np.abs(ref).max()),
                cpu_baseline=dict(entries_per_s=cpu, cores=threads, kind="port",
                                  sample="8x8-pair PDE cross Grams, oracle/pde/sigpde_oracle.c (OpenMP, same scheme)"))


def row_kuf(reps, cpu_s, increments):
    import torch
    import gpsig_amd
    from oracle import kernels_ref as kr
    T, n, l, d, m = 512, 4096, 100, 5, 5
    lt = m * (m + 1) // 2
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(2)
    Znp = rng.standard_normal((lt, T, 2, d) if increments else (lt, T, d)).astype(np.float32)
    Xnp = walks(n, l, d, 0)
    Z = torch.as_tensor(Znp, device=dev)
    X = torch.as_tensor(Xnp.reshape(n, -1), device=dev)
    k = gpsig_amd.SignatureRBF(l * d, d, m)
    fn = lambda: k.K_tens_vs_seq(Z, X, increments=increments)
    t = timed(fn, reps)
    kms = kernel_ms(fn)
    got = k.K_tens_vs_seq(Z[:, :8], X[:32], increments=increments).double().cpu().numpy()
    kref = kr.SignatureKernelRef(l * d, d, m)
    ref = kref.K_tens_vs_seq(Znp[:, :8].astype(np.float64), Xnp[:32].reshape(32, -1).astype(np.float64),
                             increments=increments)
    b_entry = 4 * lt * l * (1 + int(increments)) + 4 * (m + 1)
    Zc, Xc = Znp[:, :4].astype(np.float64), Xnp[:4].reshape(4, -1).astype(np.float64)
    cpu = cpu_rate(lambda: kref.K_tens_vs_seq(Zc, Xc, increments=increments), 16, cpu_s)
    return dict(config="C4" + ("i" if increments else ""),
                workload=f"Kuf K_tens_vs_seq normalised T={T} N={n} L={l} D={d} M={m} increments={increments}",
                entries_per_s=T * n / t, ms_per_call=t * 1e3, call_ms_events=kms,
                roofline=dict(bytes_per_entry=b_entry, pairs_per_launch=T * n,
                              achieved_GBs=T * n * b_entry / (kms / 1e3) / 1e9,
                              frac=T * n * b_entry / (kms / 1e3) / 1e9 / HBM_PEAK_GBS),
                max_abs_err=float(np.abs(got - ref).max()), max_abs_ref=float(np.abs(ref).max()),
                cpu_baseline=dict(entries_per_s=cpu, cores=1, kind="port",
                                  sample="4x4 (tensor, sequence) blocks, oracle/kernels_ref.py fp64 NumPy"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", default="C2,C3,C4,C4i,C5")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--cpu-seconds", type=float, default=5.0)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    res = []
    for r in args.rows.split(","):
        if r == "C2":
            o = row_gram("C2", 1024, 100, 5, 5, args.reps, args.cpu_seconds)
        elif r == "C5":
            o = row_gram("C5-1gpu", 8192, 128, 8, 6, max(2, args.reps // 2), args.cpu_seconds)
        elif r == "W46":
            o = row_gram("W46", 1024, 136, 46, 4, args.reps, args.cpu_seconds)
        elif r == "W126":
            o = row_gram("W126", 1024, 128, 126, 4, args.reps, args.cpu_seconds)
        elif r == "C3":
            o = row_pde(args.reps, args.cpu_seconds)
        elif r == "P128":
            o = row_pde(args.reps, args.cpu_seconds, n=256, l=100, d=128, dy=1, name="P128")
        elif r in ("C4", "C4i"):
            o = row_kuf(args.reps, args.cpu_seconds, r == "C4i")
        else:
            raise SystemExit(f"unknown row {r}")
        print(json.dumps(o), flush=True)
        res.append(o)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
