"""Generate the committed golden fixtures (tests/golden/*.npz).

Run in the build container (needs /root/reference only for the Cython pins):
    python tests/golden/make_golden.py

Every fixture holds float64 inputs and float64 expected outputs from the CPU oracle (oracle/), which
restates the reference line by line.  Before writing, the oracle is pinned:
  * against exact Chen-identity signatures (oracle/chen.py, the esig-equivalent check of reference
    notebooks/signature_kernel.ipynb) for order == num_levels with the linear base kernel,
    tensor-vs-sequence and tensor-vs-tensor;
  * against the reference's own Cython PDE solver (gpsig/sigKer_fast.pyx, built from its sources
    into oracle/_ref/ by oracle/build_ref.py) for the PDE diagonal grids -- the expected PDE grids
    stored in pde_diag.npz ARE the reference's outputs.
Seeds are fixed; the data follow SURVEY.md 8d (random walks scaled by 1/sqrt(L*D)) except where a
fixture deliberately uses rough i.i.d. points (the notebook's np.random.randn setting).
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import chen, pde, sigalgs  # noqa: E402
from oracle import kernels_ref as kr  # noqa: E402


def walk(rng, n, l, d):
    return np.cumsum(rng.standard_normal((n, l, d)), axis=1) / np.sqrt(l * d)


def save(name, **arrays):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **arrays)
    print(f"{name}: {os.path.getsize(path) / 1024:.1f} KiB")


def pin(cond, msg):
    if not cond:
        raise SystemExit(f"oracle pin failed: {msg}")


def main():
    # ------------------------------------------------------------------ F1: SignatureRBF K (config 1 sized)
    rng = np.random.default_rng(0)
    N, L, D, M = 64, 50, 3, 4
    X = walk(rng, N, L, D)
    X2 = walk(np.random.default_rng(1), 24, 40, D)
    k = kr.SignatureKernelRef(L * D, D, M)
    Xf, X2f = X.reshape(N, -1), X2.reshape(24, -1)
    kn = kr.SignatureKernelRef(L * D, D, M, normalization=False)
    save("rbf_gram.npz", X=X, X2=X2, num_levels=M,
         K=k.K(Xf), K_levels=k.K(Xf, return_levels=True),
         K_cross=k.K(Xf, X2f), K_cross_levels=k.K(Xf, X2f, return_levels=True),
         K_raw=kn.K_seq(k.scale_sequences(X)), Kdiag_raw=kn.K_seq_diag(k.scale_sequences(X)),
         Kdiag_unnorm=kn.Kdiag(Xf), Kdiag_norm=k.Kdiag(Xf))

    # rough data (notebook setting: i.i.d. normal points) + lengthscales / variances
    rng = np.random.default_rng(7)
    Xr = rng.standard_normal((12, 20, 3)) * 0.7
    kr2 = kr.SignatureKernelRef(60, 3, 4, lengthscales=[0.8, 1.3, 1.1], variances=[1.0, 0.5, 2.0, 1.5, 0.7])
    save("rbf_rough.npz", X=Xr, lengthscales=kr2.lengthscales, variances=kr2.variances, num_levels=4,
         K_levels=kr2.K(Xr.reshape(12, -1), return_levels=True))

    # ------------------------------------------------------------------ F2: SignatureLinear order=M vs Chen
    rng = np.random.default_rng(2)
    N, L, D, M = 16, 20, 3, 5
    X = rng.standard_normal((N, L, D))
    kl = kr.SignatureKernelRef(L * D, D, M, base="linear", order=M, normalization=False)
    Klev = kl.K_seq(X)
    Kchen = chen.signature_levels_kernel(X, X, M)
    err = np.abs(Klev - Kchen).max() / np.abs(Kchen).max()
    pin(err < 1e-12, f"linear order=M vs Chen {err}")
    save("linear_chen.npz", X=X, num_levels=M, K_levels=Klev, K_chen=Kchen)

    # ------------------------------------------------------------------ F3: higher order (RBF and linear)
    rng = np.random.default_rng(3)
    N, L, D, M = 8, 20, 3, 4
    X = walk(rng, N, L, D)
    out = {"X": X, "num_levels": M}
    for order in (2, 3, 4):
        out[f"rbf_order{order}"] = kr.SignatureKernelRef(L * D, D, M, order=order, normalization=False).K_seq(X)
        out[f"lin_order{order}"] = kr.SignatureKernelRef(L * D, D, M, base="linear", order=order,
                                                         normalization=False).K_seq(X)
    save("higher_order.npz", **out)

    # ------------------------------------------------------------------ F4: tensors
    rng = np.random.default_rng(4)
    N, L, D, M, T = 8, 20, 3, 5, 8
    X = rng.standard_normal((N, L, D)) * 0.5
    LT = M * (M + 1) // 2
    Z = rng.standard_normal((LT, T, D))
    Zi = rng.standard_normal((LT, T, 2, D)) * 0.5
    kl = kr.SignatureKernelRef(L * D, D, M, base="linear", order=M, normalization=False)
    tvs = kl.K_tens_vs_seq_raw(Z, X)
    tens = chen.simple_tensors(Z, M)
    SX = [chen.signature(x, M) for x in X]
    ref = np.stack([tens[m] @ np.stack([s[m] for s in SX]).T for m in range(M + 1)])
    pin(np.abs(tvs - ref).max() / np.abs(ref).max() < 1e-12, "tens_vs_seq vs Chen")
    tg = kl.K_tens_raw(Z)
    reft = np.stack([tens[m] @ tens[m].T for m in range(M + 1)])
    pin(np.abs(tg - reft).max() / np.abs(reft).max() < 1e-12, "tensor gram vs Chen")
    out = {"X": X, "Z": Z, "Zi": Zi, "num_levels": M, "lin_tvs_order5": tvs, "lin_tens": tg}
    for base in ("rbf", "linear"):
        for order in (1, 2, M):
            kk = kr.SignatureKernelRef(L * D, D, M, base=base, order=order, normalization=False)
            out[f"{base}_tvs_o{order}"] = kk.K_tens_vs_seq_raw(Z * 0.3, X)
            out[f"{base}_tvs_incr_o{order}"] = kk.K_tens_vs_seq_raw(Zi, X, increments=True)
        kk = kr.SignatureKernelRef(L * D, D, M, base=base, normalization=False)
        out[f"{base}_tens"] = kk.K_tens_raw(Z * 0.3)
        out[f"{base}_tens_incr"] = kk.K_tens_raw(Zi, increments=True)
    kn = kr.SignatureKernelRef(L * D, D, M)
    out["rbf_Kuf_norm_levels"] = kn.K_tens_vs_seq(Z * 0.3, X.reshape(N, -1), return_levels=True)
    save("tensors.npz", **out)

    # ------------------------------------------------------------------ F5: VOSF rescaled
    rng = np.random.default_rng(5)
    N, L, D, M, T = 4, 12, 3, 4, 3
    X = rng.standard_normal((N, L, D)) * 0.6
    Zl = np.abs(rng.standard_normal((M * (M + 1) // 2, T, D)))
    kl = kr.SignatureKernelRef(L * D, D, M, base="linear", normalization=False)
    R = kl.mahalanobis_raw(Zl, X)
    lam = chen.simple_tensors(Zl, M)
    naive = np.zeros((M + 1, N, T))
    for n, x in enumerate(X):
        S = chen.signature(x, M)
        for m in range(1, M + 1):
            for t in range(T):
                naive[m, n, t] = np.sum(S[m] * S[m]) - np.sum(S[m] * lam[m][t] * S[m])
    pin(np.abs(R - naive).max() / np.abs(naive).max() < 1e-12, "rescaled vs naive")
    # per-coordinate RBF embedding variant (kernels_pde.py:191-222)
    Zc = np.concatenate([Zl, np.ones_like(Zl)], axis=1)
    diffs = X[:, :, None, :] - X[:, None, :, :]                      # (N,L,L,D)
    E = np.exp(-diffs ** 2 / 2.0)
    Mr = np.einsum("npqd,rtd->nprtq", E, Zc)
    R_rbf = sigalgs.signature_kern_rescaled_higher_order(Mr, M)
    save("rescaled.npz", X=X, Z=Zl, num_levels=M, K_linear=R, K_naive=naive, K_rbf=R_rbf)

    # ------------------------------------------------------------------ F6: PDE (reference Cython pins)
    rng = np.random.default_rng(6)
    A, L, D = 8, 20, 3
    X = walk(rng, A, L, D) * 3.0
    out = {"X": X}
    from oracle import build_ref
    ref = build_ref.load()
    if ref is None:
        raise SystemExit("reference Cython solver unavailable; PDE fixtures need /root/reference")
    for n in (0, 1, 2):
        for solver in (0, 1):
            K, Kr = ref.sig_kern_diag(X, n, solver)
            K2, Kr2 = pde.pde_diag_grids(X, n, solver)
            tril = np.tril(np.ones(K.shape[1:], bool))
            pin(np.array_equal(K[:, tril], K2[:, tril]) and np.array_equal(Kr[:, tril], Kr2[:, tril]),
                f"C oracle vs reference Cython n={n} solver={solver}")
            out[f"diag_n{n}_s{solver}"] = K[:, -1, -1]
            if n < 2:
                out[f"grid_n{n}_s{solver}"] = K
                out[f"gridrev_n{n}_s{solver}"] = Kr
    Y = walk(np.random.default_rng(8), 5, 15, D) * 3.0
    for n in (0, 1):
        out[f"cross_n{n}"] = pde.pde_gram(X, Y, n, 1)
        out[f"sym_n{n}"] = pde.pde_gram(X, None, n, 1)
    out["Y"] = Y
    save("pde.npz", **out)

    # ------------------------------------------------------------------ F7: lags
    rng = np.random.default_rng(9)
    N, L, D, M = 10, 25, 2, 3
    X = walk(rng, N, L, D)
    out = {"X": X, "num_levels": M}
    for nl in (1, 2):
        kk = kr.SignatureKernelRef(L * D, D, M, num_lags=nl)
        out[f"lags{nl}_K_levels"] = kk.K(X.reshape(N, -1), return_levels=True)
        out[f"lags{nl}_scaled"] = kk.scale_sequences(X)
    save("lags.npz", **out)

    # ------------------------------------------------------------------ F8: difference=False
    rng = np.random.default_rng(10)
    N, L, D, M = 8, 16, 3, 3
    X = walk(rng, N, L, D)
    out = {"X": X, "num_levels": M}
    for base in ("rbf", "linear"):
        kk = kr.SignatureKernelRef(L * D, D, M, base=base, difference=False, normalization=False)
        out[f"{base}_nodiff"] = kk.K_seq(X)
    save("nodiff.npz", **out)


if __name__ == "__main__":
    main()
