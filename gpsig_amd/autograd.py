"""torch.autograd bindings of the gfx950 Gram kernels.

The reference differentiates SignatureKernel.K / Kdiag with TF autodiff through the materialised
graph (gpsig/kernels.py:209-238, 402-477, 510-541; gpsig/signature_algs.py:8-35).  Here the forward
is the fused Gram kernel and the backward is the gpsig_sig_gram_vjp kernel (gpsig_amd/csrc/sig_bwd.h):

  K(X) / K(X, X2), normalised:  out = sum_m s_m (K_m + jitter [a == b]) rs_m(a) rs_m(b)
    one VJP launch over the Gram pairs gives dLoss/dX, dLoss/dX2 through K_m, dLoss/drs and
    dLoss/ds; dLoss/drs is chained through rs = (K_m(a, a) + jitter)^-1/2 into one VJP launch over the
    diagonal pairs.

When a gradient is needed, the forward Gram launch also saves its end-of-sweep state
(gpsig_sig_gram_state: (M-1)(L2-1) + M floats per pair) and the VJP launch skips its own forward
sweep; above GRAM_STATE_BYTES (env GPSIG_GRAM_STATE_BYTES) the VJP recomputes it instead.  The Kuf state
and the PDE fronts work the same way.  All such buffers alive at once (one per autograd node between
its forward and backward: an SVGP step holds Kuu, Kuf and the Kff diagonal together) share one budget,
SAVED_STATE_BYTES (env GPSIG_SAVED_STATE_BYTES, default 32 GiB of the 288 GB HBM): a forward that would
exceed it saves nothing and its backward recomputes.

Gradients reach the sequences (and, through the host-side scaling in kernels.py, the lengthscales)
and sigma * variances.  Supported for order == 1 (difference True or False); for order > 1 the Gram and
its diagonal through gpsig_sig_gram_vjp_ho (csrc/sig_ho_bwd.h, sig_ho_bwd_lds.h: min(order, M) = 2..5,
lengths <= 512, and 6 at 6 levels up to 256 points, where the row state fits the LDS; up to 1017 points at
orders 2-5 with a global-memory slab)
and, beyond it, for SignatureLinear with order >= num_levels (the exact signature kernel; backward
through the signature features, ops.sig_gram_ho_vjp); other higher orders evaluate forward but raise
NotImplementedError on backward.  The RBF higher order past 32 channels takes its cells from the matrix-core
producer, whose LDS image of one sequence bounds d to about 180 channels at 129-160 points and about 240
otherwise (include/gpsig_amd.h, gpsig_sig_workspace_bytes_ex): past that the forward raises GpsigError.
"""
from __future__ import annotations

import os
import threading
import weakref

import torch

from . import _lib as L
from . import ops


GRAM_STATE_BYTES = int(os.environ.get("GPSIG_GRAM_STATE_BYTES", 16 << 30))
SAVED_STATE_BYTES = int(os.environ.get("GPSIG_SAVED_STATE_BYTES", 32 << 30))
_saved = {"bytes": 0}
_saved_lock = threading.Lock()


def _release_saved(nbytes):
    with _saved_lock:
        _saved["bytes"] -= nbytes


def saved_state_bytes() -> int:
    """Bytes of forward-saved VJP state (Gram state, Kuf state, PDE fronts) currently alive."""
    return _saved["bytes"]


def _saved_buffer(numel: int, device, cap: int):
    """A float32 buffer for a forward launch's saved VJP state, or None when it is larger than its kind's
    cap or would take the saved buffers alive at once past SAVED_STATE_BYTES (the backward recomputes).
    The budget is returned when the buffer is freed (after the backward, or with its autograd node)."""
    nbytes = numel * 4
    if numel <= 0 or nbytes > cap:
        return None
    with _saved_lock:
        if _saved["bytes"] + nbytes > SAVED_STATE_BYTES:
            return None
        _saved["bytes"] += nbytes
    t = torch.empty(numel, dtype=torch.float32, device=device)
    weakref.finalize(t, _release_saved, nbytes)
    return t


def _ho_signature_case(cfg):
    """Higher order with the linear base kernel and order >= num_levels (the exact signature kernel,
    as benchmarks/models/train_gpsig_vosf.py:102 trains it): differentiable through signature features."""
    return cfg["order"] >= cfg["num_levels"] and cfg["base"] in ("linear", "lin") and cfg["difference"]


def _ho_vjp_kernel(cfg, *lengths):
    """Higher order, and the higher-order VJP kernel (gpsig_sig_gram_vjp_ho) covers the sequences."""
    return (cfg["order"] > 1 and cfg["num_levels"] > 1 and cfg["difference"]
            and cfg["base"] in ("rbf", "linear", "lin")
            and all(ops.ho_vjp_supported(l, cfg["num_levels"], cfg["order"], cfg["base"]) for l in lengths))


def _channel_counts(v, d, m):
    """sum_w v_w n_c(w) for a level-m vector v (d^m, iisignature's first-index-major word order: index = w_1 d^(m-1)
    + ... + w_m) and n_c(w) the occurrences of channel c in w: per word position, the sums of v over the other
    positions, added up (no d^m x d count matrix)."""
    t = v.reshape((d,) * m)
    out = torch.zeros(d, dtype=v.dtype, device=v.device)
    for k in range(m):
        out += t.sum(dim=tuple(a for a in range(m) if a != k)) if m > 1 else t
    return out


SCALING_FEATURE_BYTES = int(os.environ.get("GPSIG_SCALING_FEATURE_BYTES", 1 << 28))


def _scaling_closed_form(cfg, Xs, X2s=None):
    """The exact signature kernel, and its fp64 signature features within SCALING_FEATURE_BYTES (beyond it the
    VJP's own gradient stands: d^M features per sequence make the closed form cost more than it saves)."""
    if not _ho_signature_case(cfg):
        return False
    d, M = Xs.shape[-1], cfg["num_levels"]
    n = Xs.shape[0] + (0 if X2s is None else X2s.shape[0])
    ln = max(Xs.shape[1], 1 if X2s is None else X2s.shape[1])
    ch = sum(d ** m for m in range(1, M + 1))
    # the features themselves and one sequence's step exponentials in _signature64 (three live copies)
    return 8 * n * ch <= SCALING_FEATURE_BYTES and 24 * max(ln - 1, 1) * ch <= SCALING_FEATURE_BYTES


def _signature64(X, M):
    """fp64 truncated signatures (n, sum_m d^m) of X (n, l, d), levels 1..M first-index-major: each step's
    tensor exponential, then Chen's identity S(a * b)_m = sum_k S(a)_k (x) S(b)_(m-k) over a pairwise tree
    (log2 l rounds), rows in chunks within SCALING_FEATURE_BYTES.  (The fp32 signature kernel's ~3e-7 relative
    error would be amplified by the cancellation the contraction below exists to avoid.)"""
    n, l, d = X.shape
    ch = sum(d ** m for m in range(1, M + 1))
    out = torch.zeros((n, ch), dtype=torch.float64, device=X.device)
    if l < 2 or n == 0:
        return out
    rows = max(1, SCALING_FEATURE_BYTES // (3 * 8 * (l - 1) * ch))
    for r0 in range(0, n, rows):
        dx = (X[r0:r0 + rows, 1:] - X[r0:r0 + rows, :-1]).double()
        E = [None, dx]
        for m in range(2, M + 1):
            E.append((E[-1][..., :, None] * dx[..., None, :]).flatten(-2) / m)
        while E[1].shape[1] > 1:
            if E[1].shape[1] % 2:  # a zero step: its exponential is the identity
                E = [None] + [torch.cat([e, torch.zeros_like(e[:, :1])], 1) for e in E[1:]]
            A = [None] + [e[:, 0::2] for e in E[1:]]
            B = [None] + [e[:, 1::2] for e in E[1:]]
            E = [None] + [A[m] + B[m] + sum((A[k][..., :, None] * B[m - k][..., None, :]).flatten(-2)
                                            for k in range(1, m)) for m in range(1, M + 1)]
        out[r0:r0 + rows] = torch.cat([e[:, 0] for e in E[1:]], -1)
    return out


def _scaling_contraction(Xs, X2s, M, gK, gd1=None, gd2=None):
    """e_c = sum_i x_ic dL/dx_ic (+ the same over X2) for the exact signature kernel (linear, order >= M), in
    closed form.  Scaling channel c of every sequence by s multiplies each level-m signature coordinate S_w by
    s^n_c(w) (n_c(w): occurrences of c in the word w), so with K_m(a, b) = <S_m(x_a), S_m(y_b)>,
        e_c = sum_m 2 sum_w n_c(w) [ sum_ab gK_m(a, b) S_w(x_a) S_w(y_b) + sum_a gd1_m(a) S_w(x_a)^2
                                      + sum_b gd2_m(b) S_w(y_b)^2 ]
    from fp64 signatures (_signature64) and one fp64 GEMM per level.  gK (M+1, n1, n2) = dL/d(raw levels)
    (for K(X) over both slots of every pair), gd1 / gd2 (M+1, n) = dL/d(raw diagonals)."""
    d = Xs.shape[-1]
    S1 = _signature64(Xs.detach(), M)
    S2 = S1 if X2s is None else _signature64(X2s.detach(), M)
    e = torch.zeros(d, dtype=torch.float64, device=Xs.device)
    off = 0
    for m in range(1, M + 1):
        w = d ** m
        P, Q = S1[:, off:off + w], S2[:, off:off + w]
        v = (P * (gK[m].double() @ Q)).sum(0)
        if gd1 is not None:
            v = v + (gd1[m].double()[:, None] * P * P).sum(0)
        if gd2 is not None:
            v = v + (gd2[m].double()[:, None] * Q * Q).sum(0)
        e += 2.0 * _channel_counts(v, d, m)
        off += w
    return e


def _project_scaling(e, Xs, gX, X2s=None, gY=None):
    """Adjust the gradient(s) along each channel's scaling direction x_c -> (1 + t) x_c so that their
    contraction sum_i x_ic g_ic equals e_c (_scaling_contraction), leaving every orthogonal component as the
    kernels computed it.  That contraction is what the lengthscale gradient reads (dL/dl_c = -e_c / l_c); over
    the points it cancels (for the normalised kernel sum_c e_c = 0 exactly), so the fp32 VJP's ~1e-6 errors
    along it would read as ~1e-5 of the lengthscale gradient.  Returns float64 gradients."""
    X = Xs.detach().double()
    gX = gX.double()
    cur = (X * gX).sum(dim=(0, 1))
    nrm = (X * X).sum(dim=(0, 1))
    if gY is not None:
        Y = X2s.detach().double()
        gY = gY.double()
        cur = cur + (Y * gY).sum(dim=(0, 1))
        nrm = nrm + (Y * Y).sum(dim=(0, 1))
    t = torch.where(nrm > 0, (e - cur) / torch.clamp(nrm, min=1e-300), torch.zeros_like(nrm))
    gX = gX + X * t
    if gY is not None:
        gY = gY + Y * t
    return gX, gY


def _check_bwd(cfg, gram=False):
    """The VJP kernels cover order 1 (difference True or False); Gram / diagonal gradients of higher
    orders are covered by the higher-order VJP kernel (checked by the caller) or, beyond it, for the
    exact signature kernel (linear, order >= num_levels)."""
    if cfg["order"] != 1 and not (gram and _ho_signature_case(cfg)):
        raise NotImplementedError("gradients of the signature kernels are implemented for order=1 "
                                  "(gpsig_sig_gram_vjp, gpsig_tens_vs_seq_vjp), for the Gram and its diagonal "
                                  "at min(order, num_levels) in 2..5 up to length 512 (1017 at fewer levels) and 6 at 6 "
                                  "levels up to 256 (gpsig_sig_gram_vjp_ho), "
                                  "and for SignatureLinear with order >= num_levels")


def _ho_gram_backward(ctx, gout):
    """Backward of SigGram for the higher-order signature case: the fused epilogue (jitter, 1/sqrt(diag)
    normalisation, sigma * variances, level sum) is restated in torch on the raw levels and differentiated
    there; the raw levels and diagonals go through ops.sig_gram_ho_vjp."""
    cfg = ctx.cfg
    Xs, X2s, sc32, rs1, rs2 = ctx.saved_tensors
    M = cfg["num_levels"]
    sym = X2s is None
    kw = dict(order=cfg["order"], base=cfg["base"], difference=cfg["difference"])
    with torch.enable_grad():
        Kr = ops.sig_gram(Xs.detach(), None if sym else X2s.detach(), M, **kw).double().requires_grad_(True)
        sc = sc32.double().requires_grad_(True)
        ins = [Kr, sc]
        if cfg["normalization"] and sym:  # kernels.py:431-434: K += jitter I, divide by its diagonal
            n = Kr.shape[1]
            Kj = Kr + cfg["jitter"] * torch.eye(n, dtype=Kr.dtype, device=Kr.device)[None]
            dd = torch.sqrt(torch.diagonal(Kj, dim1=1, dim2=2))
            K = Kj / (dd[:, :, None] * dd[:, None, :])
        elif cfg["normalization"]:  # kernels.py:457-470: the two raw diagonals + jitter
            d1 = ops.sig_diag(Xs.detach(), M, **kw).double().requires_grad_(True)
            d2 = ops.sig_diag(X2s.detach(), M, **kw).double().requires_grad_(True)
            ins += [d1, d2]
            K = Kr / (torch.sqrt(d1 + cfg["jitter"])[:, :, None] * torch.sqrt(d2 + cfg["jitter"])[:, None, :])
        else:
            K = Kr
        K = K * sc[:, None, None]
        out = K if cfg["return_levels"] else K.sum(0)
        grads = torch.autograd.grad(out, ins, gout.double())
    gK, gsc = grads[0], grads[1]
    gd1 = grads[2] if len(grads) > 2 else None
    gd2 = grads[3] if len(grads) > 3 else None
    gX, gY = ops.sig_gram_ho_vjp(Xs.detach(), None if sym else X2s.detach(), M, gK, gd1, gd2)
    gXo = gX.to(Xs.dtype) if ctx.needs_input_grad[0] else None
    gYo = gY.to(X2s.dtype) if (not sym and ctx.needs_input_grad[1]) else None
    gso = gsc.to(ctx.scale_dtype) if ctx.needs_input_grad[2] else None
    return gXo, gYo, gso, None


def _epilogue(Kr, sc, cfg):
    """The normalisation epilogue of K(X) (kernels.py:431-434: jitter, division by the square roots of the
    diagonal, sigma * variances, level sum) on raw levels, in the dtype of Kr."""
    n = Kr.shape[1]
    Kj = Kr + cfg["jitter"] * torch.eye(n, dtype=Kr.dtype, device=Kr.device)[None]
    dd = torch.sqrt(torch.diagonal(Kj, dim1=1, dim2=2))
    K = Kj / (dd[:, :, None] * dd[:, None, :]) * sc[:, None, None]
    return K if cfg["return_levels"] else K.sum(0)


def _folded(cfg, X2s, lengths, needs_grad):
    """Normalised K whose backward folds the normalisation's diagonal terms into the weights of the diagonal
    pairs (one VJP launch, see SigGram.backward): the forward keeps the raw levels (and, for K(X, X2), the raw
    diagonals).  Order 1: symmetric K(X); higher orders: under the higher-order VJP kernel, K(X) and K(X, X2)."""
    if not (needs_grad and cfg["normalization"]):
        return False
    if cfg["order"] == 1 or cfg["num_levels"] == 1:
        return X2s is None
    return _ho_vjp_kernel(cfg, *lengths)


FOLD_WEIGHT_BYTES = int(os.environ.get("GPSIG_FOLD_WEIGHT_BYTES", 1 << 30))


def _fold_blocks(n1, n2, M, budget=None):
    """Row / column block sizes of the folded K(X, X2) backward.  One upper-triangle launch over the whole
    concatenation [X; X2] evaluates (n1 + n2)^2 / 2 pairs for the n1 n2 of the X-X2 block and its (M+1)
    (n1 + n2)^2 fp64 weights: fine while the two sides are comparable (at most 2x the pairs) and the weights
    fit `budget`; otherwise the larger side (or both) is cut into blocks of about the smaller side, at least
    128 rows, so every launch carries at most ~2x its useful pairs and its weights stay within the budget."""
    budget = FOLD_WEIGHT_BYTES if budget is None else budget
    per = 12 * (M + 1)  # fp64 weights + their fp32 copy, per pair slot
    if max(n1, n2) <= 2 * min(n1, n2) and per * (n1 + n2) ** 2 <= budget:
        return n1, n2
    b = max(min(n1, n2), 128)
    b = max(1, min(b, int((budget / per) ** 0.5) // 2))
    return min(n1, b), min(n2, b)


def _epilogue_cross(Kr, d1, d2, sc, cfg):
    """kernels.py:457-470: K(X, X2) over the square roots of the two raw diagonals + jitter, sigma * variances."""
    K = Kr / (torch.sqrt(d1 + cfg["jitter"])[:, :, None] * torch.sqrt(d2 + cfg["jitter"])[:, None, :])
    K = K * sc[:, None, None]
    return K if cfg["return_levels"] else K.sum(0)


def _pad_last(X, length):
    """Sequences padded to `length` points by repeating their last point: zero increments, so every signature
    kernel value of a difference seed is unchanged."""
    n, l, d = X.shape
    return X if l == length else torch.cat([X, X[:, -1:].expand(n, length - l, d)], 1)


def _unpad_grad(g, l):
    """Gradient of the padded sequences -> of the originals (the repeats are copies of the last point)."""
    out = g[:, :l].clone()
    out[:, l - 1] += g[:, l:].sum(1)
    return out


class SigGram(torch.autograd.Function):
    """Normalised / raw signature Gram (SignatureKernel.K) with a gfx950 backward."""

    @staticmethod
    def forward(ctx, Xs, X2s, scale, cfg):
        M = cfg["num_levels"]
        lengths = (Xs.shape[1],) if X2s is None else (max(Xs.shape[1], X2s.shape[1]),)
        if _folded(cfg, X2s, lengths, any(ctx.needs_input_grad[:3])):
            # raw levels (and diagonals) from the kernels, the epilogue in fp64 (the backward differentiates it)
            kw = dict(order=cfg["order"], base=cfg["base"], difference=cfg["difference"])
            state = None
            if cfg["order"] == 1 and cfg["difference"]:  # the VJP then skips its forward sweep
                numel = ops.sig_state_numel(Xs.shape[0], None, Xs.shape[1], M)
                state = _saved_buffer(numel, Xs.device, GRAM_STATE_BYTES)
            Kr = ops.sig_gram(Xs.detach(), None if X2s is None else X2s.detach(), M, state=state, **kw)
            sc32 = scale.detach().to(torch.float32)
            ctx.cfg = cfg
            ctx.scale_dtype = scale.dtype
            ctx.state = state
            ctx.folded = True
            if X2s is None:
                ctx.save_for_backward(Xs, X2s, sc32, Kr, None, None)
                return _epilogue(Kr.double(), sc32.double(), cfg).to(torch.float32)
            d1 = ops.sig_diag(Xs.detach(), M, **kw)
            d2 = ops.sig_diag(X2s.detach(), M, **kw)
            ctx.save_for_backward(Xs, X2s, sc32, Kr, d1, d2)
            return _epilogue_cross(Kr.double(), d1.double(), d2.double(), sc32.double(), cfg).to(torch.float32)
        ctx.folded = False
        mode = L.OUT_NORM_LEVELS if cfg["return_levels"] else L.OUT_NORM_SUM
        sc32 = scale.detach().to(torch.float32)
        kw = dict(order=cfg["order"], base=cfg["base"], difference=cfg["difference"])
        rs1 = rs2 = None
        if cfg["normalization"]:
            rs1 = ops.sig_diag(Xs.detach(), M, jitter=cfg["jitter"], rsqrt=True, **kw)
            rs2 = rs1 if X2s is None else ops.sig_diag(X2s.detach(), M, jitter=cfg["jitter"], rsqrt=True, **kw)
        jit = cfg["jitter"] if (cfg["normalization"] and X2s is None) else 0.0
        state = None
        if any(ctx.needs_input_grad[:3]) and cfg["order"] == 1 and cfg["difference"]:
            n2 = None if X2s is None else X2s.shape[0]
            numel = ops.sig_state_numel(Xs.shape[0], n2, Xs.shape[1] if X2s is None else X2s.shape[1], M)
            state = _saved_buffer(numel, Xs.device, GRAM_STATE_BYTES)
        out = ops.sig_gram(Xs.detach(), None if X2s is None else X2s.detach(), M, rs1=rs1, rs2=rs2, scale=sc32,
                           jitter=jit, out_mode=mode, state=state, **kw)
        ctx.state = state
        ctx.cfg = cfg
        ctx.scale_dtype = scale.dtype
        ctx.save_for_backward(Xs, X2s, sc32, rs1, rs2)
        return out

    @staticmethod
    def backward(ctx, gout):
        cfg = ctx.cfg
        if ctx.folded:
            # dLoss/dK_m(a, b) of the epilogue in fp64, the diagonal's own term (through 1/sqrt(K_m(a, a)))
            # included in the weight of the pair (a, a): ONE VJP launch over the upper triangle.  The diagonal
            # term's direction is the pair (a, a)'s own derivative, so its large part cancels in the scalar
            # weight; computed as separate Gram and diagonal VJPs the two terms cancel ~270x at the VOSF
            # trainer's shape and their fp32 rounding dominated the gradient.
            Xs, X2s, sc32, Kr, d1, d2 = ctx.saved_tensors
            vjp = dict(base=cfg["base"], gout_levels=True, difference=cfg["difference"], order=cfg["order"])
            M = cfg["num_levels"]
            if X2s is None:
                with torch.enable_grad():
                    K64 = Kr.double().requires_grad_(True)
                    sc = sc32.double().requires_grad_(True)
                    gK, gsc = torch.autograd.grad(_epilogue(K64, sc, cfg), [K64, sc], gout.double())
                gX, _ = ops.sig_gram_vjp(Xs.detach(), None, M, gK.to(torch.float32), state=ctx.state, **vjp)
                ctx.state = None
                if _scaling_closed_form(cfg, Xs):  # the scaling directions in closed form (lengthscale gradients)
                    gX, _ = _project_scaling(_scaling_contraction(Xs, None, M, gK), Xs, gX)
                return (gX.to(Xs.dtype) if ctx.needs_input_grad[0] else None, None,
                        gsc.to(ctx.scale_dtype) if ctx.needs_input_grad[2] else None, None)
            # K(X, X2): the Gram pairs and both sets of diagonal pairs in ONE upper-triangle launch over the
            # concatenation [X; X2] (padded to a common length by repeating last points), the weights in blocks:
            # dLoss/dK(a, b) on the X-X2 block, the diagonal terms on the diagonal, nothing else (those pairs exit
            # at once, sig_ho_bwd_lds.h)
            with torch.enable_grad():
                K64, D1, D2 = (t.double().requires_grad_(True) for t in (Kr, d1, d2))
                sc = sc32.double().requires_grad_(True)
                gK, g1, g2, gsc = torch.autograd.grad(_epilogue_cross(K64, D1, D2, sc, cfg), [K64, D1, D2, sc],
                                                      gout.double())
            n1, l1 = Xs.shape[:2]
            n2, l2 = X2s.shape[:2]
            lm = max(l1, l2)
            Xp = _pad_last(Xs.detach().to(torch.float32), lm)
            X2p = _pad_last(X2s.detach().to(torch.float32), lm)
            gX = torch.zeros(Xp.shape, dtype=torch.float64, device=Xs.device)
            gY = torch.zeros(X2p.shape, dtype=torch.float64, device=Xs.device)
            b1, b2 = _fold_blocks(n1, n2, M)
            # one launch per block pair (rows r of X, rows c of X2) over [X_r; X2_c]: the X-X2 weights of the
            # block, X_r's diagonal terms in the first column block, X2_c's in the first row block
            for r0 in range(0, n1, b1):
                r1 = min(n1, r0 + b1)
                for c0 in range(0, n2, b2):
                    c1 = min(n2, c0 + b2)
                    m1, m2 = r1 - r0, c1 - c0
                    Gc = torch.zeros((M + 1, m1 + m2, m1 + m2), dtype=torch.float64, device=Xs.device)
                    Gc[:, :m1, m1:] = gK[:, r0:r1, c0:c1]
                    if c0 == 0:
                        i1 = torch.arange(m1, device=Xs.device)
                        Gc[:, i1, i1] = g1[:, r0:r1]
                    if r0 == 0:
                        i2 = torch.arange(m1, m1 + m2, device=Xs.device)
                        Gc[:, i2, i2] = g2[:, c0:c1]
                    gXc, _ = ops.sig_gram_vjp(torch.cat([Xp[r0:r1], X2p[c0:c1]]), None, M, Gc.to(torch.float32), **vjp)
                    gX[r0:r1] += gXc[:m1]
                    gY[c0:c1] += gXc[m1:]
            gX, gY = _unpad_grad(gX, l1), _unpad_grad(gY, l2)
            if _scaling_closed_form(cfg, Xs, X2s):
                gX, gY = _project_scaling(_scaling_contraction(Xs, X2s, M, gK, g1, g2), Xs, gX, X2s, gY)
            return (gX.to(Xs.dtype) if ctx.needs_input_grad[0] else None,
                    gY.to(X2s.dtype) if ctx.needs_input_grad[1] else None,
                    gsc.to(ctx.scale_dtype) if ctx.needs_input_grad[2] else None, None)
        Xs, X2s, sc32, rs1, rs2 = ctx.saved_tensors
        lengths = (Xs.shape[1],) if X2s is None else (Xs.shape[1], X2s.shape[1])
        if cfg["order"] != 1 and not _ho_vjp_kernel(cfg, *lengths):
            _check_bwd(cfg, gram=True)
            return _ho_gram_backward(ctx, gout)
        order = cfg["order"]
        M = cfg["num_levels"]
        sym = X2s is None
        dev = Xs.device
        n1 = Xs.shape[0]
        n2 = n1 if sym else X2s.shape[0]
        grs1 = grs2 = None
        if cfg["normalization"]:
            grs1 = torch.zeros((M + 1, n1), dtype=torch.float32, device=dev)
            grs2 = grs1 if sym else torch.zeros((M + 1, n2), dtype=torch.float32, device=dev)
        gscale = torch.zeros((M + 1,), dtype=torch.float32, device=dev)
        jit = cfg["jitter"] if (cfg["normalization"] and sym) else 0.0
        gX, gY = ops.sig_gram_vjp(Xs.detach(), None if sym else X2s.detach(), M, gout, base=cfg["base"],
                                  difference=cfg["difference"], order=order,
                                  gout_levels=cfg["return_levels"], rs1=rs1, rs2=rs2, scale=sc32, jitter=jit,
                                  grs1=grs1, grs2=grs2, gscale=gscale, state=ctx.state)
        ctx.state = None
        if cfg["normalization"]:
            # rs = (K_m(a, a) + jitter)^-1/2  ->  dLoss/dK_m(a, a) = -rs^3/2 dLoss/drs
            ops.sig_gram_vjp(Xs.detach(), None, M, grs1 * (-0.5) * rs1 ** 3, base=cfg["base"], diag=True, gX=gX,
                             difference=cfg["difference"], order=order)
            if not sym:
                ops.sig_gram_vjp(X2s.detach(), None, M, grs2 * (-0.5) * rs2 ** 3, base=cfg["base"], diag=True,
                                 difference=cfg["difference"], order=order, gX=gY)
        if _scaling_closed_form(cfg, Xs, X2s) and not cfg["normalization"]:
            # unnormalised: dL/dK_m(raw) = gout (per level, or summed) times sigma * variances_m
            g = gout.double() if cfg["return_levels"] else gout.double()[None].expand(M + 1, -1, -1)
            gK = g * sc32.double()[:, None, None]
            gX, gY = _project_scaling(_scaling_contraction(Xs, X2s, M, gK), Xs, gX, X2s, None if sym else gY)
        gXo = gX.to(Xs.dtype) if ctx.needs_input_grad[0] else None
        gYo = gY.to(X2s.dtype) if (not sym and ctx.needs_input_grad[1]) else None
        gso = gscale.to(ctx.scale_dtype) if ctx.needs_input_grad[2] else None
        return gXo, gYo, gso, None


class SigDiag(torch.autograd.Function):
    """Raw per-level diagonal k(x_a, x_a) (SignatureKernel._K_seq_diag) with a gfx950 backward."""

    @staticmethod
    def forward(ctx, Xs, cfg):
        ctx.cfg = cfg
        ctx.save_for_backward(Xs)
        return ops.sig_diag(Xs.detach(), cfg["num_levels"], cfg["order"], cfg["base"], cfg["difference"])

    @staticmethod
    def backward(ctx, gout):
        cfg = ctx.cfg
        (Xs,) = ctx.saved_tensors
        if cfg["order"] != 1 and not _ho_vjp_kernel(cfg, Xs.shape[1]):
            _check_bwd(cfg, gram=True)
            gX, _ = ops.sig_gram_ho_vjp(Xs.detach(), None, cfg["num_levels"], None, gout)
        else:
            gX, _ = ops.sig_gram_vjp(Xs.detach(), None, cfg["num_levels"], gout, base=cfg["base"], diag=True,
                                     difference=cfg["difference"], order=cfg["order"])
        return gX.to(Xs.dtype), None


class TensVsSeq(torch.autograd.Function):
    """Raw per-level inducing-tensor vs sequence kernel (SignatureKernel._K_tens_vs_seq) with a gfx950
    backward (gpsig_tens_vs_seq_vjp) for dLoss/dZ and dLoss/dX."""

    @staticmethod
    def forward(ctx, Zs, Xs, cfg):
        ctx.cfg = cfg
        ctx.save_for_backward(Zs, Xs)
        ctx.state = None
        args = (Zs.detach(), Xs.detach(), cfg["num_levels"], cfg["order"], cfg["base"], cfg["difference"],
                cfg["increments"])
        numel = ops.tens_state_numel(Zs.shape[1], Xs.shape[0], cfg["num_levels"])
        st = None
        if any(ctx.needs_input_grad[:2]) and cfg["order"] == 1 and cfg["difference"]:
            st = _saved_buffer(numel, Xs.device, GRAM_STATE_BYTES)
        if st is not None:
            # the training step keeps the forward's end state: the VJP skips its forward sweep
            out, ctx.state = ops.tens_vs_seq(*args, state=st)
            return out
        return ops.tens_vs_seq(*args)

    @staticmethod
    def backward(ctx, gout):
        cfg = ctx.cfg
        _check_bwd(cfg)  # gpsig_tens_vs_seq_vjp differentiates the order-1 recursion only
        Zs, Xs = ctx.saved_tensors
        gZ, gX = ops.tens_vs_seq_vjp(Zs.detach(), Xs.detach(), cfg["num_levels"], gout, cfg["base"],
                                     cfg["increments"], difference=cfg["difference"], state=ctx.state)
        ctx.state = None
        return (gZ.to(Zs.dtype) if ctx.needs_input_grad[0] else None,
                gX.to(Xs.dtype) if ctx.needs_input_grad[1] else None, None)


class TensGram(torch.autograd.Function):
    """Raw per-level inducing-tensor Gram (SignatureKernel._K_tens) with a gfx950 backward
    (gpsig_tens_gram_vjp) for dLoss/dZ."""

    @staticmethod
    def forward(ctx, Zs, cfg):
        ctx.cfg = cfg
        ctx.save_for_backward(Zs)
        return ops.tens_gram(Zs.detach(), cfg["num_levels"], cfg["base"], cfg["increments"])

    @staticmethod
    def backward(ctx, gout):
        cfg = ctx.cfg
        (Zs,) = ctx.saved_tensors
        gZ = ops.tens_gram_vjp(Zs.detach(), cfg["num_levels"], gout, cfg["base"], cfg["increments"])
        return gZ.to(Zs.dtype), None


PDE_FRONTS_BYTES = int(os.environ.get("GPSIG_PDE_FRONTS_BYTES", 16 << 30))


def _pde_fronts_buffer(ctx, Xs, npairs, l1, l2, dyadic):
    """Buffer for the PDE adjoint's forward fronts when a gradient is needed and they fit
    PDE_FRONTS_BYTES (env GPSIG_PDE_FRONTS_BYTES); None: the backward recomputes them."""
    if not any(ctx.needs_input_grad[:2]):
        return None
    nb = ops.pde_fronts_bytes(npairs, l1, l2, dyadic)
    return _saved_buffer((nb + 3) // 4, Xs.device, PDE_FRONTS_BYTES) if nb else None


class PdeDiag(torch.autograd.Function):
    """k(x_a, x_a) of the Goursat PDE (UntruncSignatureKernel.Kdiag) with the reference's adjoint
    (kernels_pde.py:465-509) as backward (gpsig_pde_vjp, DIAG)."""

    @staticmethod
    def forward(ctx, Xs, dyadic, solver):
        ctx.dyadic, ctx.solver = dyadic, solver
        ctx.save_for_backward(Xs)
        ctx.fronts = _pde_fronts_buffer(ctx, Xs, Xs.shape[0], Xs.shape[1], Xs.shape[1], dyadic)
        if ctx.fronts is not None:  # the training step's forward keeps the adjoint's fronts
            return ops.pde_fronts(Xs.detach(), None, dyadic, solver, ctx.fronts, diag=True)
        return ops.pde_diag(Xs.detach(), dyadic, solver)

    @staticmethod
    def backward(ctx, gout):
        (Xs,) = ctx.saved_tensors
        if ctx.fronts is not None:
            gX = ops.pde_vjp_fronts(Xs.detach(), None, gout, ctx.dyadic, ctx.solver, ctx.fronts, diag=True)
            ctx.fronts = None
        else:
            gX = ops.pde_diag_vjp(Xs.detach(), gout, ctx.dyadic, ctx.solver)
        return gX.to(Xs.dtype), None, None


class PdeGram(torch.autograd.Function):
    """PDE cross Gram (UntruncSignatureKernel.K) with the same adjoint extended to cross pairs."""

    @staticmethod
    def forward(ctx, Xs, X2s, dyadic, solver):
        ctx.dyadic, ctx.solver = dyadic, solver
        ctx.save_for_backward(Xs, X2s)
        Y = Xs if X2s is None else X2s
        ctx.fronts = _pde_fronts_buffer(ctx, Xs, Xs.shape[0] * Y.shape[0], Xs.shape[1], Y.shape[1], dyadic)
        X2d = None if X2s is None else X2s.detach()
        if ctx.fronts is not None:  # the training step's forward keeps the adjoint's fronts
            return ops.pde_fronts(Xs.detach(), X2d, dyadic, solver, ctx.fronts)
        return ops.pde_gram(Xs.detach(), X2d, dyadic, solver)

    @staticmethod
    def backward(ctx, gout):
        Xs, X2s = ctx.saved_tensors
        X2d = None if X2s is None else X2s.detach()
        if ctx.fronts is not None:
            gX, gY = ops.pde_vjp_fronts(Xs.detach(), X2d, gout, ctx.dyadic, ctx.solver, ctx.fronts)
            ctx.fronts = None
        else:
            gX, gY = ops.pde_gram_vjp(Xs.detach(), X2d, gout, ctx.dyadic, ctx.solver)
        return (gX.to(Xs.dtype), None if gY is None else gY.to(X2s.dtype), None, None)


class Signature(torch.autograd.Function):
    """Truncated signatures (iisignature.sig) with the gfx950 backward (iisignature.sigbackprop)."""

    @staticmethod
    def forward(ctx, X, depth):
        ctx.depth = depth
        ctx.save_for_backward(X)
        return ops.signature(X.detach(), depth)

    @staticmethod
    def backward(ctx, gout):
        (X,) = ctx.saved_tensors
        return ops.signature_vjp(X.detach(), ctx.depth, gout).to(X.dtype), None
