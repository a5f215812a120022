#!/usr/bin/env python
"""Forward vs forward+backward time of the differentiable paths on one GPU (median of --reps
device-synchronised calls, inputs resident), with the gradient's error vs torch fp64 autodiff of the
reference graph (oracle/autodiff_ref.py) / the reference's PDE adjoint (oracle/pde_grad.py) on a
subsample.  One JSON object per line.

    python tools/bench_grad.py [--only gram,kuf,kuf_incr,pde,pde_gram,sig,svgp46,svgp126]
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


def walks(n, l, d, seed):
    rng = np.random.default_rng(seed)
    return np.cumsum(rng.standard_normal((n, l, d)), axis=1) / np.sqrt(l * d)


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts)


def rel(g, r):
    return float(np.abs(g - r).max() / np.abs(r).max())


def bench_gram(reps, n=1024, l=100, d=5, m=5):
    import gpsig_amd
    from oracle import autodiff_ref as ar
    Xnp = walks(n, l, d, 0)
    X = torch.tensor(Xnp.reshape(n, -1), device="cuda", dtype=torch.float32)
    G = torch.randn(n, n, device="cuda")
    k = gpsig_amd.SignatureRBF(l * d, d, m)

    def fwd():
        with torch.no_grad():
            k.K(X)

    def fb():
        Xg = X.detach().requires_grad_(True)
        (k.K(Xg) * G).sum().backward()

    tf, tb = timed(fwd, reps), timed(fb, reps)
    S = 8
    Xs = torch.tensor(Xnp[:S].reshape(S, -1), device="cuda", requires_grad=True)
    Gs = torch.randn(S, S, dtype=torch.float64)
    (k.K(Xs) * Gs.to("cuda")).sum().backward()
    Xr = torch.tensor(Xnp[:S], requires_grad=True)
    (ar.K(Xr, None, m) * Gs).sum().backward()
    return dict(path="gram", workload=f"SignatureRBF K(X) normalised N={n} L={l} D={d} M={m}", fwd_ms=tf * 1e3,
                fwd_bwd_ms=tb * 1e3, grad_err=rel(Xs.grad.reshape(Xr.shape).cpu().numpy(), Xr.grad.numpy()))


def bench_kuf(reps, t=512, n=1024, l=100, d=5, m=5, increments=False):
    import gpsig_amd
    from oracle import autodiff_ref as ar
    lt = m * (m + 1) // 2
    rng = np.random.default_rng(2)
    Znp = rng.standard_normal((lt, t, 2, d) if increments else (lt, t, d))
    Xnp = walks(n, l, d, 0)
    Z = torch.tensor(Znp, device="cuda", dtype=torch.float32)
    X = torch.tensor(Xnp.reshape(n, -1), device="cuda", dtype=torch.float32)
    G = torch.randn(t, n, device="cuda")
    k = gpsig_amd.SignatureRBF(l * d, d, m)

    def fwd():
        with torch.no_grad():
            k.K_tens_vs_seq(Z, X, increments=increments)

    def fb():
        Zg = Z.detach().requires_grad_(True)
        (k.K_tens_vs_seq(Zg, X, increments=increments) * G).sum().backward()

    tf, tb = timed(fwd, reps), timed(fb, reps)
    S, TS = 6, 5
    Zs = torch.tensor(Znp[:, :TS], device="cuda", requires_grad=True)
    Gs = torch.randn(TS, S, dtype=torch.float64)
    (k.K_tens_vs_seq(Zs, torch.tensor(Xnp[:S].reshape(S, -1), device="cuda"), increments=increments)
     * Gs.to("cuda")).sum().backward()
    Zr = torch.tensor(Znp[:, :TS], requires_grad=True)
    (ar.K_tens_vs_seq(Zr, torch.tensor(Xnp[:S]), m, increments=increments) * Gs).sum().backward()
    return dict(path="kuf" + ("_incr" if increments else ""),
                workload=f"K_tens_vs_seq normalised T={t} N={n} L={l} D={d} M={m} increments={increments} (dZ)",
                fwd_ms=tf * 1e3, fwd_bwd_ms=tb * 1e3, grad_err=rel(Zs.grad.cpu().numpy(), Zr.grad.numpy()))


def bench_pde(reps, n=1024, l=200, d=5, dyadic=1):
    import gpsig_amd
    from oracle import pde, pde_grad
    Xnp = walks(n, l, d, 0)
    X = torch.tensor(Xnp.reshape(n, -1), device="cuda", dtype=torch.float32)
    w = torch.randn(n, device="cuda")
    k = gpsig_amd.UntruncSignatureKernel(l * d, d, order=dyadic)

    def fwd():
        with torch.no_grad():
            k.Kdiag(X)

    def fb():
        Xg = X.detach().requires_grad_(True)
        (k.Kdiag(Xg) * w).sum().backward()

    tf, tb = timed(fwd, reps), timed(fb, reps)
    S = 4
    Xs = torch.tensor(Xnp[:S].reshape(S, -1), device="cuda", requires_grad=True)
    k.Kdiag(Xs).sum().backward()
    K, Kr = pde.pde_diag_grids(Xnp[:S], dyadic, 1)
    ref = pde_grad.kdiag_grad(Xnp[:S], np.tril(K), np.tril(Kr), dyadic)
    return dict(path="pde_kdiag", workload=f"UntruncSignatureKernel Kdiag N={n} L={l} D={d} dyadic={dyadic}",
                fwd_ms=tf * 1e3, fwd_bwd_ms=tb * 1e3, grad_err=rel(Xs.grad.reshape(ref.shape).cpu().numpy(), ref))


def bench_pde_gram(reps, n=256, l=100, d=5, dyadic=1):
    """PDE cross Gram K(X, X2) (new in this build; the reference has only Kdiag) and its VJP."""
    import gpsig_amd
    from oracle import pde_grad
    Xnp, Ynp = walks(n, l, d, 0), walks(n, l, d, 1)
    X = torch.tensor(Xnp.reshape(n, -1), device="cuda", dtype=torch.float32)
    Y = torch.tensor(Ynp.reshape(n, -1), device="cuda", dtype=torch.float32)
    G = torch.randn(n, n, device="cuda")
    k = gpsig_amd.UntruncSignatureKernel(l * d, d, order=dyadic)

    def fwd():
        with torch.no_grad():
            k.K(X, Y)

    def fb():
        Xg = X.detach().requires_grad_(True)
        (k.K(Xg, Y) * G).sum().backward()

    tf, tb = timed(fwd, reps), timed(fb, reps)
    Xs = torch.tensor(Xnp[:1].reshape(1, -1), device="cuda", requires_grad=True)
    Ys = torch.tensor(Ynp[:1].reshape(1, -1), device="cuda")
    k.K(Xs, Ys).sum().backward()
    ref, _ = pde_grad.pair_grad(Xnp[0], Ynp[0], dyadic)
    return dict(path="pde_gram", workload=f"UntruncSignatureKernel K(X, X2) N={n}x{n} L={l} D={d} dyadic={dyadic} (dX)",
                fwd_ms=tf * 1e3, fwd_bwd_ms=tb * 1e3, grad_err=rel(Xs.grad.reshape(ref.shape).cpu().numpy(), ref))


def bench_sig(reps, n=4096, l=100, d=5, depth=3):
    from gpsig_amd import signatures as sg
    from oracle import autodiff_ref as ar
    Xnp = walks(n, l, d, 0)
    X = torch.tensor(Xnp, device="cuda", dtype=torch.float32)
    C = sum(d ** m for m in range(1, depth + 1))
    G = torch.randn(n, C, device="cuda")

    def fwd():
        with torch.no_grad():
            sg.Sig(X, depth)

    def fb():
        Xg = X.detach().requires_grad_(True)
        (sg.Sig(Xg, depth) * G).sum().backward()

    tf, tb = timed(fwd, reps), timed(fb, reps)
    xs = torch.tensor(Xnp[0], requires_grad=True)
    Xg = torch.tensor(Xnp[:1], device="cuda", requires_grad=True)
    g0 = torch.randn(C, dtype=torch.float64)
    (sg.Sig(Xg, depth) * g0.to("cuda")[None]).sum().backward()
    (ar.signature(xs, depth) * g0).sum().backward()
    return dict(path="signature", workload=f"Sig N={n} L={l} d={d} depth={depth}", fwd_ms=tf * 1e3,
                fwd_bwd_ms=tb * 1e3, grad_err=rel(Xg.grad[0].cpu().numpy(), xs.grad.numpy()))


def bench_svgp(reps, t=500, n=50, l=500, nf=23, m=4):
    """One SVGP training step's kernel bundle at the reference runner's shapes
    (benchmarks/run_gpsig_benchmarks.py:32 -> models/train_gpsig.py:20-58): SignatureRBF(num_levels=4,
    num_lags=1, add_time) with InducingTensors(num_inducing=500, increments=True), a minibatch of 50
    sequences of max_len 500; nf raw features + time, so D = 2 nf after the lag (46 AUSLAN, 126 CMU).
    Kuu_Kuf_Kff (inducing_variables.py:51-67) forward, then the backward to Z, the lengthscales and the
    variances (X is data).  The gradient paths are parity-tested in tests/ (test_wide_gpu, test_training_gpu);
    this row is timing only."""
    import gpsig_amd
    from gpsig_amd.inducing_variables import InducingTensors
    D = 2 * nf
    lt = m * (m + 1) // 2
    rng = np.random.default_rng(5)
    Xnp = walks(n, l, nf, 0)
    X = torch.tensor(Xnp.reshape(n, -1), device="cuda", dtype=torch.float64)
    Z0 = torch.tensor(rng.standard_normal((lt, t, 2, D)) * 0.3, device="cuda", dtype=torch.float64)
    k = gpsig_amd.SignatureRBF(l * nf, nf, m, num_lags=1, lengthscales=np.ones(nf))
    k.to("cuda")
    Gzz = torch.randn(t, t, device="cuda", dtype=torch.float64)
    Gzx = torch.randn(t, n, device="cuda", dtype=torch.float64)
    Gxx = torch.randn(n, device="cuda", dtype=torch.float64)

    def step(grad):
        feat = InducingTensors(Z0.detach().requires_grad_(grad), m, increments=True)
        if grad:
            for v in (k.lengthscales, k.variances):
                v.requires_grad_(True)
                v.grad = None
        with torch.set_grad_enabled(grad):
            Kzz, Kzx, Kxx = feat.Kuu_Kuf_Kff(k, X, jitter=1e-6)
            if grad:
                ((Kzz * Gzz).sum() + (Kzx * Gzx).sum() + (Kxx * Gxx).sum()).backward()

    tf, tb = timed(lambda: step(False), reps), timed(lambda: step(True), reps)
    for v in (k.lengthscales, k.variances):
        v.requires_grad_(False)
    return dict(path=f"svgp_d{D}", workload=f"SVGP step Kuu_Kuf_Kff SignatureRBF num_levels={m} num_lags=1 D={D} "
                f"InducingTensors T={t} increments=True, minibatch N={n} L={l} (dZ, dlengthscales, dvariances)",
                fwd_ms=tf * 1e3, fwd_bwd_ms=tb * 1e3, grad_err=svgp_grad_err(Xnp, Z0, nf, m))


def svgp_grad_err(Xnp, Z0, nf, m, ts=16, ns=2):
    """The same bundle's gradients on a subsample (the first ts inducing tensors, ns sequences, full length
    and channel count) against fp64 autodiff of the reference graph: Kzz = tensor_kern x sigma*variances,
    Kzx normalised by the sequences' diagonals (kernels.py:624-704), the scaling and lags (kernels.py:344-399)
    restated by the kernel's own torch code on CPU float64.  Max over dZ, dlengthscales, dvariances of
    max|g - g64| / max|g64|."""
    import gpsig_amd
    from gpsig_amd.inducing_variables import InducingTensors
    from oracle import autodiff_ref as ar
    l = Xnp.shape[1]
    Z = Z0[:, :ts].detach().cpu().numpy()
    X = Xnp[:ns]
    rng = np.random.default_rng(9)
    Gzz, Gzx = rng.standard_normal((ts, ts)), rng.standard_normal((ts, ns))
    out = {}
    for dev in ("cuda", "cpu"):
        k = gpsig_amd.SignatureRBF(l * nf, nf, m, num_lags=1, lengthscales=np.ones(nf))
        k.to(dev)
        for v in (k.lengthscales, k.variances):
            v.requires_grad_(True)
        Zt = torch.tensor(Z, device=dev, requires_grad=True)
        Xt = torch.tensor(X.reshape(ns, -1), device=dev)
        if dev == "cuda":
            Kzz, Kzx, _ = InducingTensors(Zt, m, increments=True).Kuu_Kuf_Kff(k, Xt)
        else:  # fp64 reference graph on the kernel's own scaling of the same parameters
            Xs = k._prep(Xt)
            Zs = k._apply_scaling_to_incremental_tensors(Zt)
            sv = k.sigma * k.variances
            Kzz = (ar.k_tens(Zs, m, "rbf", increments=True) * sv[:, None, None]).sum(0)
            Kzx = ar.K_tens_vs_seq(Zs, Xs, m, base="rbf", increments=True, scale=sv)
        ((Kzz * torch.tensor(Gzz, device=dev)).sum() + (Kzx * torch.tensor(Gzx, device=dev)).sum()).backward()
        out[dev] = [t.grad.detach().cpu().double().numpy() for t in (Zt, k.lengthscales, k.variances)]
    return max(rel(g, r) for g, r in zip(out["cuda"], out["cpu"]))


def bench_vosf_kdiag(reps, n=50, l=500, nf=23, m=5):
    """The VOSF-truncated trainer's Kff diagonal (benchmarks/models/train_gpsig_vosf.py:102: SignatureLinear(
    num_levels=5, order=5), minibatch 50, max_len 500, add_time: d = 24) forward and backward -- the
    higher-order VJP's LDS-state kernel (csrc/sig_ho_bwd_lds.h) at W = 8, order 5."""
    import gpsig_amd
    from oracle import autodiff_ref as ar
    d = nf + 1
    Xnp = walks(n, l, d, 0)
    X = torch.tensor(Xnp.reshape(n, -1), device="cuda", dtype=torch.float32)
    G = torch.randn(n, device="cuda")
    k = gpsig_amd.SignatureLinear(l * d, d, m, order=m, normalization=False)

    def fwd():
        with torch.no_grad():
            k.Kdiag(X)

    def fb():
        Xg = X.detach().requires_grad_(True)
        (k.Kdiag(Xg) * G).sum().backward()

    tf, tb = timed(fwd, reps), timed(fb, reps)
    S = 2
    Xs = torch.tensor(Xnp[:S].reshape(S, -1), device="cuda", requires_grad=True)
    Gs = torch.randn(S, dtype=torch.float64)
    (k.Kdiag(Xs) * Gs.to("cuda")).sum().backward()
    Xr = torch.tensor(Xnp[:S], requires_grad=True)
    (ar.k_seq_diag(Xr, m, "linear", True, order=m).sum(0) * Gs).sum().backward()
    return dict(path="vosf_kdiag", workload=f"SignatureLinear(num_levels={m}, order={m}) Kdiag N={n} L={l} D={d}",
                fwd_ms=tf * 1e3, fwd_bwd_ms=tb * 1e3, grad_err=rel(Xs.grad.reshape(Xr.shape).cpu().numpy(), Xr.grad.numpy()))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--only", default="gram,kuf,kuf_incr,pde,pde_gram,sig")
    a = ap.parse_args()
    todo = a.only.split(",")
    runs = dict(gram=lambda: bench_gram(a.reps), kuf=lambda: bench_kuf(a.reps),
                kuf_incr=lambda: bench_kuf(a.reps, increments=True), pde=lambda: bench_pde(a.reps),
                pde_gram=lambda: bench_pde_gram(a.reps),
                sig=lambda: bench_sig(a.reps), svgp46=lambda: bench_svgp(a.reps, nf=23),
                svgp126=lambda: bench_svgp(a.reps, nf=63), vosf_kdiag=lambda: bench_vosf_kdiag(a.reps))
    for name in todo:
        r = runs[name]()
        r["bwd_over_fwd"] = (r["fwd_bwd_ms"] - r["fwd_ms"]) / r["fwd_ms"]
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
