"""Typed wrappers over the C ABI (include/gpsig_amd.h) for torch device tensors.

Every function here launches HIP kernels from gpsig_amd/libgpsig_amd.so on the caller's current
stream; inputs must already be on the GPU (there is no CPU path).  Workspaces are cached per device
and stream-ordered (a cached buffer is only reused by later launches on the same stream order).
"""
from __future__ import annotations

import threading

import torch

from . import _lib as L

_ws_lock = threading.Lock()
_ws: dict = {}

BASES = {"rbf": L.BASE_RBF, "gauss": L.BASE_RBF, "linear": L.BASE_LINEAR, "lin": L.BASE_LINEAR}


def _require_cuda(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise L.GpsigError("gpsig_amd kernels need GPU tensors (device='cuda'); there is no CPU fallback")


def _f32(t: torch.Tensor) -> torch.Tensor:
    return t.to(torch.float32).contiguous() if (t.dtype != torch.float32 or not t.is_contiguous()) else t


def _ptr(t):
    return None if t is None else t.data_ptr()


def _stream(device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def workspace(device, nbytes: int) -> torch.Tensor:
    key = (torch.device(device).index, torch.cuda.current_stream(device).cuda_stream)
    with _ws_lock:
        buf = _ws.get(key)
        if buf is None or buf.numel() < nbytes:
            buf = torch.empty(max(nbytes, 1 << 20), dtype=torch.uint8, device=device)
            _ws[key] = buf
        return buf


def scratch(device, nbytes: int):
    """A second per-stream cached buffer for calls that take a workspace AND a scratch (the PDE adjoint's
    fronts plus the increment tiles); None when nothing is needed."""
    if nbytes <= 0:
        return None
    key = ("scratch", torch.device(device).index, torch.cuda.current_stream(device).cuda_stream)
    with _ws_lock:
        buf = _ws.get(key)
        if buf is None or buf.numel() < nbytes:
            buf = torch.empty(max(nbytes, 1 << 20), dtype=torch.uint8, device=device)
            _ws[key] = buf
        return buf


def _sp(buf):
    return (None, 0) if buf is None else (buf.data_ptr(), buf.numel())


def release_workspaces() -> None:
    """Drop the cached per-stream scratch buffers (feature records, the PDE VJP's K_rev cells -- up to
    PDE_VJP_SCRATCH bytes); the next call allocates again.  Captured graphs (gpsig_amd.graphs) keep
    their own references to the buffers they address."""
    with _ws_lock:
        _ws.clear()


def base_kind(base) -> int:
    if isinstance(base, int):
        return base
    try:
        return BASES[base.lower()]
    except KeyError:
        raise L.GpsigError(f"base kernel {base!r} has no gfx950 kernel (supported: rbf, linear)") from None


# ----------------------------------------------------------------------------- truncated kernels
# The exact signature kernel (linear base kernel, difference=True, order >= num_levels): the higher-order
# recursion (signature_algs.py:37-74) is then exactly K_m(x, y) = <S_m(x), S_m(y)> (tests/golden/linear_chen.npz
# pins it), so the Gram is computed as truncated signatures (gpsig_signature) + one GEMM per level on the
# matrix cores (hipBLASLt fp32) instead of the O(order^2 L^2) recursion per pair -- the configuration the
# reference's VOSF / exact-signature models train (benchmarks/models/train_gpsig_vosf.py:102,
# train_gpsig_.py:62).  Up to this many signature coordinates per sequence (the signature kernel's LDS).
SIG_FEATURE_MAX = 16000


def _sig_feature_path(order: int, base, difference: bool, num_levels: int, d: int) -> bool:
    if order < num_levels or not difference or base_kind(base) != L.BASE_LINEAR:
        return False
    return 0 < int(L.load().gpsig_signature_channels(d, num_levels)) <= SIG_FEATURE_MAX


def _sig_feature_levels(S1: torch.Tensor, S2: torch.Tensor, d: int, num_levels: int) -> torch.Tensor:
    """(M+1, n1, n2): level 0 = 1, level m = S_m(x) S_m(y)^T (one fp32 GEMM per level)."""
    out = torch.empty((num_levels + 1, S1.shape[0], S2.shape[0]), dtype=torch.float32, device=S1.device)
    out[0] = 1.0
    off = 0
    for m in range(1, num_levels + 1):
        w = d ** m
        torch.matmul(S1[:, off:off + w], S2[:, off:off + w].T, out=out[m])
        off += w
    return out


def sig_diag(X: torch.Tensor, num_levels: int, order: int = 1, base="rbf", difference: bool = True,
             jitter: float = 0.0, rsqrt: bool = False) -> torch.Tensor:
    """Per-level k(x_a, x_a), (num_levels+1, n) float32 [rsqrt: 1/sqrt(k + jitter)]."""
    _require_cuda(X)
    lib = L.load()
    X = _f32(X)
    n, l, d = X.shape
    out = torch.empty((num_levels + 1, n), dtype=torch.float32, device=X.device)
    if n == 0:  # an empty batch: empty output, as the reference's graph
        return out
    if _sig_feature_path(order, base, difference, num_levels, d):
        S = signature(X, num_levels)
        out[0] = 1.0
        off = 0
        for m in range(1, num_levels + 1):
            w = d ** m
            out[m] = (S[:, off:off + w] ** 2).sum(1)
            off += w
        return torch.rsqrt(out + float(jitter)) if rsqrt else out
    nb = lib.gpsig_sig_workspace_bytes_ex(n, l, n, l, d, order, L.PAIRS_DIAG)
    ws = workspace(X.device, nb)
    rc = lib.gpsig_sig_diag(X.data_ptr(), n, l, d, num_levels, order, base_kind(base), int(difference), float(jitter),
                            L.OUT_RSQRT if rsqrt else L.OUT_LEVELS, out.data_ptr(), ws.data_ptr(), ws.numel(),
                            _stream(X.device))
    L.check(rc, "gpsig_sig_diag")
    return out


def sig_gram(X: torch.Tensor, Y: torch.Tensor | None, num_levels: int, order: int = 1, base="rbf",
             difference: bool = True, rows: tuple | None = None, rs1=None, rs2=None, scale=None,
             jitter: float = 0.0, out_mode: int = L.OUT_LEVELS, out: torch.Tensor | None = None,
             out_row0: int | None = None, state: torch.Tensor | None = None) -> torch.Tensor:
    """Signature-kernel Gram between the sequences of X (n1,l1,d) and Y (n2,l2,d).

    Y is None -> symmetric K(X): only b >= a is evaluated and mirrored.  rows=(r0, r1) restricts the
    evaluated rows (row sharding); the output then holds rows [out_row0, out_row0 + out.shape[-2]).
    out_mode: L.OUT_LEVELS (raw per level), L.OUT_NORM_LEVELS, L.OUT_NORM_SUM (fused normalisation).
    state: float32 buffer of sig_state_numel(...) elements -> also save the VJP's forward state
    (gpsig_sig_gram_state; order 1, difference=True).
    """
    _require_cuda(X, Y, rs1, rs2, scale)
    lib = L.load()
    X = _f32(X)
    sym = Y is None
    Y = X if sym else _f32(Y)
    n1, l1, d = X.shape
    n2, l2, d2 = Y.shape
    if d2 != d:
        raise ValueError("X and Y must have the same channel count")
    r0, r1 = (0, n1) if rows is None else rows
    if out_row0 is None:
        out_row0 = r0
    if out is None:
        nrows = r1 - out_row0
        shape = (nrows, n2) if out_mode == L.OUT_NORM_SUM else (num_levels + 1, nrows, n2)
        out = torch.empty(shape, dtype=torch.float32, device=X.device)
    out_rows = out.shape[-2]
    if n1 == 0 or n2 == 0 or r1 == r0:  # an empty batch
        return out
    if state is None and _sig_feature_path(order, base, difference, num_levels, d):
        # the exact signature kernel: signatures + per-level GEMMs, then the fused epilogue's arithmetic
        S1 = signature(X[r0:r1], num_levels)
        S2 = signature(Y, num_levels)
        K = _sig_feature_levels(S1, S2, d, num_levels)
        if out_mode != L.OUT_LEVELS:
            if sym and jitter:
                idx = torch.arange(r0, r1, device=X.device)
                K[:, idx - r0, idx] += float(jitter)
            if rs1 is not None:
                K = K * _f32(rs1)[:, r0:r1, None] * _f32(rs2)[:, None, :]
            if scale is not None:
                K = K * _f32(scale)[:, None, None]
        if out_mode == L.OUT_NORM_SUM:
            K = K.sum(0)
        out[..., r0 - out_row0:r1 - out_row0, :] = K
        if sym and rows is None:  # k(x_a, x_b) = k(x_b, x_a) exactly, as the mirrored kernel output
            out.copy_(torch.triu(out) + torch.triu(out, 1).transpose(-1, -2))
        return out
    if rs1 is not None:
        rs1, rs2 = _f32(rs1), _f32(rs2)
    if scale is not None:
        scale = _f32(scale)
    pm = L.PAIRS_UPPER if sym else L.PAIRS_RECT
    nb = lib.gpsig_sig_workspace_bytes_ex(n1, l1, n2, l2, d, order, pm)
    if base_kind(base) & L.GRAM_SPLIT:  # split diagnostic: one chunk of pairs' cells in the workspace
        nb += lib.gpsig_sig_split_bytes(l1, l2, d, num_levels)
    ws = workspace(X.device, nb)
    if state is not None:
        if order != 1 or not difference:
            raise ValueError("the saved VJP state needs order=1 and difference=True")
        if state.dtype != torch.float32 or not state.is_contiguous() or state.device != X.device:
            raise ValueError("state must be a contiguous float32 tensor on the input's device")
        rc = lib.gpsig_sig_gram_state(X.data_ptr(), n1, l1, Y.data_ptr(), n2, l2, d, num_levels, base_kind(base),
                                      pm, r0, r1, _ptr(rs1), _ptr(rs2), _ptr(scale), float(jitter), out_mode,
                                      out.data_ptr(), out_row0, out_rows, state.data_ptr(), state.numel() * 4,
                                      ws.data_ptr(), ws.numel(), _stream(X.device))
        L.check(rc, "gpsig_sig_gram_state")
        return out
    rc = lib.gpsig_sig_gram(X.data_ptr(), n1, l1, Y.data_ptr(), n2, l2, d, num_levels, order, base_kind(base),
                            int(difference), pm, r0, r1,
                            _ptr(rs1), _ptr(rs2), _ptr(scale), float(jitter), out_mode, out.data_ptr(),
                            out_row0, out_rows, ws.data_ptr(), ws.numel(), _stream(X.device))
    L.check(rc, "gpsig_sig_gram")
    return out


def sig_state_numel(n1: int, n2: int | None, l2: int, num_levels: int) -> int:
    """float32 elements of the saved VJP state of a Gram call (n2 None: symmetric K(X), upper
    triangle)."""
    lib = L.load()
    sym = n2 is None
    nb = lib.gpsig_sig_state_bytes(n1, n1 if sym else n2, l2, num_levels, L.PAIRS_UPPER if sym else L.PAIRS_RECT)
    return nb // 4


def sig_gram_vjp(X: torch.Tensor, Y: torch.Tensor | None, num_levels: int, gout: torch.Tensor, base="rbf",
                 gout_levels: bool = False, diag: bool = False, rs1=None, rs2=None, scale=None, jitter: float = 0.0,
                 gX: torch.Tensor | None = None, gY: torch.Tensor | None = None, grs1=None, grs2=None,
                 gscale=None, rows: tuple | None = None, state: torch.Tensor | None = None,
                 difference: bool = True, order: int = 1):
    """dLoss/dX (and dLoss/dY, dLoss/drs, dLoss/dscale) of the Gram, accumulated into float32 buffers: see
    gpsig_sig_gram_vjp (order 1) and gpsig_sig_gram_vjp_ho (order > 1) in include/gpsig_amd.h.  Y None ->
    symmetric K(X) (or the diagonal with diag=True; gout is then (num_levels+1, n) per level).  state: the
    buffer a sig_gram(..., state=) call on the same inputs filled -> the forward sweep is skipped (order 1).
    Returns (gX, gY)."""
    _require_cuda(X, Y, gout, rs1, rs2, scale)
    lib = L.load()
    X = _f32(X)
    sym = Y is None
    Y = X if sym else _f32(Y)
    n1, l1, d = X.shape
    n2, l2, d2 = Y.shape
    if d2 != d:
        raise ValueError("X and Y must have the same channel count")
    gout = _f32(gout)
    if diag:
        if not sym:
            raise ValueError("diag=True needs Y=None")
        if tuple(gout.shape) != (num_levels + 1, n1):
            raise ValueError(f"diagonal gout must be (num_levels+1, n) = {(num_levels + 1, n1)}")
        gout_levels = True
    else:
        want = (num_levels + 1, n1, n2) if gout_levels else (n1, n2)
        if tuple(gout.shape) != want:
            raise ValueError(f"gout must have shape {want}, got {tuple(gout.shape)}")
    r0, r1 = (0, n1) if rows is None else rows
    if state is not None and diag:
        raise ValueError("the saved state is for Gram (RECT / UPPER) calls, not diag=True")
    if gX is None:
        gX = torch.zeros((n1, l1, d), dtype=torch.float32, device=X.device)
    if not sym and gY is None:
        gY = torch.zeros((n2, l2, d), dtype=torch.float32, device=X.device)
    for t, shp in ((gX, (n1, l1, d)), (gY, None if sym else (n2, l2, d))):
        if shp is not None and (t.dtype != torch.float32 or not t.is_contiguous() or tuple(t.shape) != shp):
            raise ValueError(f"gradient buffers must be contiguous float32 {shp}")
    if rs1 is not None:
        rs1, rs2 = _f32(rs1), _f32(rs2)
    if scale is not None:
        scale = _f32(scale)
    mode = L.PAIRS_DIAG if diag else (L.PAIRS_UPPER if sym else L.PAIRS_RECT)
    if order > 1 and num_levels > 1:
        if state is not None or not difference:
            raise ValueError("the higher-order VJP takes difference=True and no saved state")
        nb = lib.gpsig_sig_vjp_ho_workspace_bytes(n1, l1, n2, l2, d, num_levels, order, base_kind(base))
        if nb == 0:
            L.check(L.GPSIG_EUNSUPPORTED, f"gpsig_sig_gram_vjp_ho (order {order}, num_levels {num_levels}, "
                                          f"length {l2})")
        ws = workspace(X.device, nb)
        rc = lib.gpsig_sig_gram_vjp_ho(X.data_ptr(), n1, l1, Y.data_ptr(), n2, l2, d, num_levels, order,
                                       base_kind(base), mode, r0, r1, gout.data_ptr(), int(bool(gout_levels)),
                                       _ptr(rs1), _ptr(rs2), _ptr(scale), float(jitter), gX.data_ptr(), _ptr(gY),
                                       _ptr(grs1), _ptr(grs2), _ptr(gscale), ws.data_ptr(), ws.numel(),
                                       _stream(X.device))
        L.check(rc, "gpsig_sig_gram_vjp_ho")
        return gX, gY
    nb = lib.gpsig_sig_vjp_workspace_bytes(n1, l1, n2, l2, d, num_levels, int(bool(difference)))
    ws = workspace(X.device, nb)
    rc = lib.gpsig_sig_gram_vjp(X.data_ptr(), n1, l1, Y.data_ptr(), n2, l2, d, num_levels, base_kind(base),
                                int(bool(difference)), mode, r0, r1,
                                gout.data_ptr(), int(bool(gout_levels)), _ptr(rs1), _ptr(rs2), _ptr(scale),
                                float(jitter), gX.data_ptr(), _ptr(gY), _ptr(grs1), _ptr(grs2), _ptr(gscale),
                                _ptr(state), ws.data_ptr(), ws.numel(), _stream(X.device))
    L.check(rc, "gpsig_sig_gram_vjp")
    return gX, gY


# ----------------------------------------------------------------------------- PDE kernel
def pde_diag(X: torch.Tensor, dyadic: int = 0, solver: int = 1) -> torch.Tensor:
    _require_cuda(X)
    lib = L.load()
    X = _f32(X)
    n, l, d = X.shape
    out = torch.empty((n,), dtype=torch.float32, device=X.device)
    if n == 0:
        return out
    sp, sb = _sp(scratch(X.device, lib.gpsig_pde_scratch_bytes(n, l, n, l, d, dyadic, L.PAIRS_DIAG)))
    L.check(lib.gpsig_pde_diag_ex(X.data_ptr(), n, l, d, dyadic, solver, out.data_ptr(), sp, sb, _stream(X.device)),
            "gpsig_pde_diag")
    return out


def pde_gram(X: torch.Tensor, Y: torch.Tensor | None = None, dyadic: int = 0, solver: int = 1,
             rows: tuple | None = None, out: torch.Tensor | None = None, out_row0: int | None = None) -> torch.Tensor:
    _require_cuda(X, Y)
    lib = L.load()
    X = _f32(X)
    sym = Y is None
    Y = X if sym else _f32(Y)
    n1, l1, d = X.shape
    n2, l2, _ = Y.shape
    r0, r1 = (0, n1) if rows is None else rows
    if out_row0 is None:
        out_row0 = r0
    if out is None:
        out = torch.empty((r1 - out_row0, n2), dtype=torch.float32, device=X.device)
    if n1 == 0 or n2 == 0 or r1 == r0:
        return out
    pm = L.PAIRS_UPPER if sym else L.PAIRS_RECT
    sp, sb = _sp(scratch(X.device, lib.gpsig_pde_scratch_bytes(n1, l1, n2, l2, d, dyadic, pm)))
    rc = lib.gpsig_pde_gram_ex(X.data_ptr(), n1, l1, Y.data_ptr(), n2, l2, d, dyadic, solver, pm, r0, r1,
                               out.data_ptr(), out_row0, out.shape[-2], sp, sb, _stream(X.device))
    L.check(rc, "gpsig_pde_gram")
    return out


PDE_VJP_SCRATCH = 4 << 30  # bytes of adjoint fronts per launch (rows are chunked to fit)


def pde_diag_vjp(X: torch.Tensor, gout: torch.Tensor, dyadic: int = 0, solver: int = 1,
                 gX: torch.Tensor | None = None) -> torch.Tensor:
    """dLoss/dX of pde_diag (the reference's _KdiagGrad adjoint, kernels_pde.py:465-509) given gout (n,)."""
    _require_cuda(X, gout)
    lib = L.load()
    X, gout = _f32(X), _f32(gout)
    n, l, d = X.shape
    if gX is None:
        gX = torch.zeros((n, l, d), dtype=torch.float32, device=X.device)
    per = lib.gpsig_pde_vjp_workspace_bytes(1, l, l, dyadic)
    step = max(1, min(n, PDE_VJP_SCRATCH // max(per, 1)))
    sp, sb = _sp(scratch(X.device, lib.gpsig_pde_vjp_scratch_bytes(n, l, n, l, d, dyadic, L.PAIRS_DIAG)))
    for r0 in range(0, n, step):
        r1 = min(n, r0 + step)
        ws = workspace(X.device, lib.gpsig_pde_vjp_workspace_bytes(r1 - r0, l, l, dyadic))
        rc = lib.gpsig_pde_vjp_ex(X.data_ptr(), n, l, X.data_ptr(), n, l, d, dyadic, solver, L.PAIRS_DIAG, r0, r1,
                                  gout.data_ptr(), gX.data_ptr(), None, ws.data_ptr(), ws.numel(), sp, sb,
                                  _stream(X.device))
        L.check(rc, "gpsig_pde_vjp")
    return gX


def pde_gram_vjp(X: torch.Tensor, Y: torch.Tensor | None, gout: torch.Tensor, dyadic: int = 0, solver: int = 1):
    """(dLoss/dX, dLoss/dY) of pde_gram given gout (n1, n2) (Y None: symmetric K(X), returns (gX, None))."""
    _require_cuda(X, Y, gout)
    lib = L.load()
    X, gout = _f32(X), _f32(gout)
    sym = Y is None
    Y = X if sym else _f32(Y)
    n1, l1, d = X.shape
    n2, l2, _ = Y.shape
    if tuple(gout.shape) != (n1, n2):
        raise ValueError(f"gout must be {(n1, n2)}")
    gX = torch.zeros((n1, l1, d), dtype=torch.float32, device=X.device)
    gY = gX if sym else torch.zeros((n2, l2, d), dtype=torch.float32, device=X.device)
    per = lib.gpsig_pde_vjp_workspace_bytes(n2, l1, l2, dyadic)
    step = max(4, (min(n1, PDE_VJP_SCRATCH // max(per, 1)) // 4) * 4)
    sp, sb = _sp(scratch(X.device, lib.gpsig_pde_vjp_scratch_bytes(n1, l1, n2, l2, d, dyadic, L.PAIRS_RECT)))
    for r0 in range(0, n1, step):
        r1 = min(n1, r0 + step)
        ws = workspace(X.device, lib.gpsig_pde_vjp_workspace_bytes((r1 - r0) * n2, l1, l2, dyadic))
        rc = lib.gpsig_pde_vjp_ex(X.data_ptr(), n1, l1, Y.data_ptr(), n2, l2, d, dyadic, solver, L.PAIRS_RECT, r0,
                                  r1, gout.data_ptr(), gX.data_ptr(), gY.data_ptr(), ws.data_ptr(), ws.numel(), sp, sb,
                                  _stream(X.device))
        L.check(rc, "gpsig_pde_vjp")
    return gX, (None if sym else gY)


def pde_fronts_bytes(n_pairs: int, l1: int, l2: int, dyadic: int) -> int:
    """Bytes of the PDE adjoint's forward fronts for n_pairs pairs (0: the adjoint does not apply)."""
    return int(L.load().gpsig_pde_vjp_workspace_bytes(n_pairs, l1, l2, dyadic))


def pde_fronts(X: torch.Tensor, Y: torch.Tensor | None, dyadic: int, solver: int, fronts: torch.Tensor,
               diag: bool = False) -> torch.Tensor:
    """Forward of a training step (gpsig_pde_fronts): the values of pde_gram(X, Y) (all n1 x n2 pairs;
    Y None: Y = X, symmetrised) or, diag=True, of pde_diag(X), and the adjoint's fronts in `fronts` (a
    float32 buffer of pde_fronts_bytes(...) / 4 elements) for pde_vjp_fronts."""
    _require_cuda(X, Y, fronts)
    lib = L.load()
    X = _f32(X)
    sym = Y is None
    Y = X if sym else _f32(Y)
    n1, l1, d = X.shape
    n2, l2, _ = Y.shape
    npairs = n1 if diag else n1 * n2
    if fronts.dtype != torch.float32 or not fronts.is_contiguous() or fronts.numel() * 4 < pde_fronts_bytes(npairs, l1, l2, dyadic):
        raise ValueError("fronts must be a contiguous float32 buffer of pde_fronts_bytes() bytes")
    out = torch.empty((n1,) if diag else (n1, n2), dtype=torch.float32, device=X.device)
    pm = L.PAIRS_DIAG if diag else L.PAIRS_RECT
    sp, sb = _sp(scratch(X.device, lib.gpsig_pde_vjp_scratch_bytes(n1, l1, n2, l2, d, dyadic, pm)))
    rc = lib.gpsig_pde_fronts_ex(X.data_ptr(), n1, l1, Y.data_ptr(), n2, l2, d, dyadic, solver, pm, 0, n1,
                                 out.data_ptr(), fronts.data_ptr(), fronts.numel() * 4, sp, sb, _stream(X.device))
    L.check(rc, "gpsig_pde_fronts")
    if sym and not diag:  # k(x_a, x_b) = k(x_b, x_a): the upper triangle mirrored, as pde_gram's
        out = torch.triu(out) + torch.triu(out, 1).T
    return out


def pde_vjp_fronts(X: torch.Tensor, Y: torch.Tensor | None, gout: torch.Tensor, dyadic: int, solver: int,
                   fronts: torch.Tensor, diag: bool = False):
    """The adjoint from the fronts a pde_fronts call on the same inputs left (gpsig_pde_vjp_fronts):
    (gX, gY) as pde_gram_vjp, or gX as pde_diag_vjp with diag=True."""
    _require_cuda(X, Y, gout, fronts)
    lib = L.load()
    X, gout = _f32(X), _f32(gout)
    sym = Y is None
    Y = X if sym else _f32(Y)
    n1, l1, d = X.shape
    n2, l2, _ = Y.shape
    gX = torch.zeros((n1, l1, d), dtype=torch.float32, device=X.device)
    gY = gX if (sym or diag) else torch.zeros((n2, l2, d), dtype=torch.float32, device=X.device)
    pm = L.PAIRS_DIAG if diag else L.PAIRS_RECT
    sp, sb = _sp(scratch(X.device, lib.gpsig_pde_vjp_scratch_bytes(n1, l1, n2, l2, d, dyadic, pm)))
    rc = lib.gpsig_pde_vjp_fronts_ex(X.data_ptr(), n1, l1, Y.data_ptr(), n2, l2, d, dyadic, solver, pm, 0, n1,
                                     gout.data_ptr(), gX.data_ptr(), None if diag else gY.data_ptr(),
                                     fronts.data_ptr(), fronts.numel() * 4, sp, sb, _stream(X.device))
    L.check(rc, "gpsig_pde_vjp_fronts")
    if diag:
        return gX
    return gX, (None if sym else gY)


# ----------------------------------------------------------------------------- signature features
def ho_vjp_supported(l2: int, num_levels: int, order: int, base="rbf") -> bool:
    """Whether gpsig_sig_gram_vjp_ho covers (length, levels, order, base kernel)."""
    return L.load().gpsig_sig_vjp_ho_workspace_bytes(1, 2, 1, l2, 1, num_levels, order, base_kind(base)) > 0


def sig_gram_ho_vjp(X: torch.Tensor, Y: torch.Tensor | None, num_levels: int, gK: torch.Tensor | None,
                    gd1: torch.Tensor | None = None, gd2: torch.Tensor | None = None):
    """dLoss/dX, dLoss/dY of the raw per-level higher-order Gram of the linear base kernel with
    order >= num_levels (signature_algs.py:37-74 over kernels.py:979-986; the configuration
    benchmarks/models/train_gpsig_vosf.py:102 trains).  There the recursion is exactly the inner product of
    truncated signatures, K_m(x, y) = <S_m(x), S_m(y)> (tests/golden/linear_chen.npz pins it), so the VJP
    goes through the signature features: dLoss/dS_m(x_a) = sum_b gK_m(a, b) S_m(y_b) (+ 2 gd1_m(a) S_m(x_a)
    for the raw diagonal), then the gfx950 signature VJP (gpsig_signature_vjp).

    gK (M+1, n1, n2) = dLoss/dK_m for K(X, Y), or for the symmetric K(X) when Y is None; gd1 (M+1, n1),
    gd2 (M+1, n2) = dLoss/d(raw diagonal) of X and Y.  Returns (gX, gY) float32 (gY None when Y is None).
    """
    M = num_levels
    X = _f32(X)
    n1, l1, d = X.shape
    PX = signature(X, M)
    sizes = [d ** m for m in range(1, M + 1)]
    offs = [sum(sizes[:m]) for m in range(M + 1)]
    PY = PX if Y is None else signature(_f32(Y), M)
    gPX = torch.zeros_like(PX)
    gPY = None if Y is None else torch.zeros_like(PY)
    for m in range(1, M + 1):
        sl = slice(offs[m - 1], offs[m])
        if gK is not None:
            g = gK[m].to(torch.float32)
            if Y is None:
                gPX[:, sl] += (g + g.T) @ PX[:, sl]
            else:
                gPX[:, sl] += g @ PY[:, sl]
                gPY[:, sl] += g.T @ PX[:, sl]
        if gd1 is not None:
            gPX[:, sl] += 2.0 * gd1[m].to(torch.float32)[:, None] * PX[:, sl]
        if gd2 is not None and Y is not None:
            gPY[:, sl] += 2.0 * gd2[m].to(torch.float32)[:, None] * PY[:, sl]
    gX = signature_vjp(X, M, gPX)
    gY = None if Y is None else signature_vjp(_f32(Y), M, gPY)
    return gX, gY


def signature(X: torch.Tensor, depth: int) -> torch.Tensor:
    """Truncated signatures, levels 1..depth flattened first-index-major (iisignature.sig layout):
    X (n, l, d) -> (n, sum_m d^m) float32."""
    _require_cuda(X)
    lib = L.load()
    X = _f32(X)
    n, l, d = X.shape
    out = torch.empty((n, int(lib.gpsig_signature_channels(d, depth))), dtype=torch.float32, device=X.device)
    if n == 0:
        return out
    ws = workspace(X.device, lib.gpsig_signature_workspace_bytes(n, d, depth, 0))  # past the LDS: level slabs
    L.check(lib.gpsig_signature_ex(X.data_ptr(), n, l, d, depth, out.data_ptr(), ws.data_ptr(), ws.numel(),
                                   _stream(X.device)), "gpsig_signature")
    return out


def signature_vjp(X: torch.Tensor, depth: int, gout: torch.Tensor, gX: torch.Tensor | None = None) -> torch.Tensor:
    """dLoss/dX of signature() given gout (n, channels) (iisignature.sigbackprop)."""
    _require_cuda(X, gout)
    lib = L.load()
    X, gout = _f32(X), _f32(gout)
    n, l, d = X.shape
    if tuple(gout.shape) != (n, int(lib.gpsig_signature_channels(d, depth))):
        raise ValueError("gout must be (n, channels)")
    if gX is None:
        gX = torch.zeros((n, l, d), dtype=torch.float32, device=X.device)
    ws = workspace(X.device, lib.gpsig_signature_workspace_bytes(n, d, depth, 1))
    L.check(lib.gpsig_signature_vjp_ex(X.data_ptr(), n, l, d, depth, gout.data_ptr(), gX.data_ptr(), ws.data_ptr(),
                                       ws.numel(), _stream(X.device)), "gpsig_signature_vjp")
    return gX


# ----------------------------------------------------------------------------- multi-GPU helper
def sym_assemble(src: torch.Tensor, row_off: torch.Tensor, level_stride: int, n: int, levels: int,
                 out: torch.Tensor | None = None) -> torch.Tensor:
    """Full symmetric (levels, n, n) from gathered UPPER-mode rows: global row a (level 0) starts at
    element row_off[a] of src, level l at + l*level_stride."""
    _require_cuda(src, row_off)
    lib = L.load()
    if src.dtype != torch.float32 or not src.is_contiguous():
        raise ValueError("src must be contiguous float32")
    row_off = row_off.to(torch.int64).contiguous()
    if out is None:
        out = torch.empty((levels, n, n), dtype=torch.float32, device=src.device)
    L.check(lib.gpsig_sym_assemble(src.data_ptr(), row_off.data_ptr(), int(level_stride), n, levels, out.data_ptr(),
                                   _stream(src.device)), "gpsig_sym_assemble")
    return out


# ----------------------------------------------------------------------------- inducing tensors
def tens_vs_seq(Z: torch.Tensor, X: torch.Tensor, num_levels: int, order: int = 1, base="rbf",
                difference: bool = True, increments: bool = False, state: torch.Tensor | None = None):
    """<z_t, S(x_n)> per level: Z (LT,T,D) or (LT,T,2,D) with increments, X (N,L,D) -> (M+1, T, N).
    state: a float32 buffer of tens_state_numel(...) elements -> also the VJP's saved state
    (gpsig_tens_vs_seq_state); returns (out, state) then, state None where the fast paths do not apply."""
    _require_cuda(Z, X)
    lib = L.load()
    Z, X = _f32(Z), _f32(X)
    lt, t, d = Z.shape[0], Z.shape[1], Z.shape[-1]
    n, l, dx = X.shape
    if dx != d:
        raise ValueError("Z and X must have the same channel count")
    if lt != num_levels * (num_levels + 1) // 2:
        raise ValueError(f"Z must have num_levels*(num_levels+1)/2 = {num_levels * (num_levels + 1) // 2} components")
    out = torch.empty((num_levels + 1, t, n), dtype=torch.float32, device=X.device)
    if n == 0 or t == 0:
        return (out, None) if state is not None else out
    ws = workspace(X.device, lib.gpsig_tens_workspace_bytes(n, l, d, lt, t))
    if state is not None:
        if state.dtype != torch.float32 or not state.is_contiguous() or state.numel() < t * n * lt:
            raise ValueError("state must be a contiguous float32 buffer of tens_state_numel() elements")
        rc = L.GPSIG_EUNSUPPORTED
        if order == 1 and difference:
            rc = lib.gpsig_tens_vs_seq_state(Z.data_ptr(), lt, t, int(increments), d, X.data_ptr(), n, l, num_levels,
                                             base_kind(base), out.data_ptr(), state.data_ptr(), ws.data_ptr(),
                                             ws.numel(), _stream(X.device))
        if rc != L.GPSIG_EUNSUPPORTED:
            L.check(rc, "gpsig_tens_vs_seq_state")
            return out, state
        return tens_vs_seq(Z, X, num_levels, order, base, difference, increments), None
    rc = lib.gpsig_tens_vs_seq(Z.data_ptr(), lt, t, int(increments), d, X.data_ptr(), n, l, num_levels, order,
                               base_kind(base), int(difference), out.data_ptr(), ws.data_ptr(), ws.numel(),
                               _stream(X.device))
    L.check(rc, "gpsig_tens_vs_seq")
    return out


def tens_state_numel(t: int, n: int, num_levels: int) -> int:
    """Floats of the tens_vs_seq VJP's saved state: (T, N, LT)."""
    return t * n * (num_levels * (num_levels + 1) // 2)


def tens_vs_seq_vjp(Z: torch.Tensor, X: torch.Tensor, num_levels: int, gout: torch.Tensor, base="rbf",
                    increments: bool = False, gZ: torch.Tensor | None = None, gX: torch.Tensor | None = None,
                    difference: bool = True, state: torch.Tensor | None = None):
    """dLoss/dZ, dLoss/dX of the raw per-level tens_vs_seq output (order 1, difference True or False) given
    gout (num_levels+1, T, N); accumulated into float32 buffers (see gpsig_tens_vs_seq_vjp)."""
    _require_cuda(Z, X, gout)
    lib = L.load()
    Z, X = _f32(Z), _f32(X)
    lt, t, d = Z.shape[0], Z.shape[1], Z.shape[-1]
    n, l, dx = X.shape
    if dx != d:
        raise ValueError("Z and X must have the same channel count")
    if tuple(gout.shape) != (num_levels + 1, t, n):
        raise ValueError(f"gout must be (num_levels+1, T, N) = {(num_levels + 1, t, n)}")
    gout = _f32(gout)
    if gZ is None:
        gZ = torch.zeros(Z.shape, dtype=torch.float32, device=Z.device)
    if gX is None:
        gX = torch.zeros(X.shape, dtype=torch.float32, device=X.device)
    nb = lib.gpsig_tens_vjp_workspace_bytes(n, l, d) if d <= 16 else lib.gpsig_tens_vjp_wide_workspace_bytes(n, l, d, lt, t)
    ws = workspace(X.device, nb)
    rc = lib.gpsig_tens_vs_seq_vjp(Z.data_ptr(), lt, t, int(increments), d, X.data_ptr(), n, l, num_levels,
                                   base_kind(base), int(bool(difference)), gout.data_ptr(), gZ.data_ptr(),
                                   gX.data_ptr(), _ptr(state), ws.data_ptr(),
                                   ws.numel(), _stream(X.device))
    L.check(rc, "gpsig_tens_vs_seq_vjp")
    return gZ, gX


def tens_gram(Z: torch.Tensor, num_levels: int, base="rbf", increments: bool = False) -> torch.Tensor:
    """Inducing-tensor Gram per level: Z (LT,T,D) or (LT,T,2,D) -> (M+1, T, T)."""
    _require_cuda(Z)
    lib = L.load()
    Z = _f32(Z)
    lt, t, d = Z.shape[0], Z.shape[1], Z.shape[-1]
    out = torch.empty((num_levels + 1, t, t), dtype=torch.float32, device=Z.device)
    nb = lib.gpsig_tens_gram_workspace_bytes(lt, t, d)
    ws = workspace(Z.device, nb) if nb else None
    rc = lib.gpsig_tens_gram(Z.data_ptr(), lt, t, int(increments), d, num_levels, base_kind(base), out.data_ptr(),
                             _ptr(ws), ws.numel() if nb else 0, _stream(Z.device))
    L.check(rc, "gpsig_tens_gram")
    return out


def tens_gram_vjp(Z: torch.Tensor, num_levels: int, gout: torch.Tensor, base="rbf", increments: bool = False,
                  gZ: torch.Tensor | None = None) -> torch.Tensor:
    """dLoss/dZ of the raw per-level tensor Gram given gout (num_levels+1, T, T) (gpsig_tens_gram_vjp)."""
    _require_cuda(Z, gout)
    lib = L.load()
    Z = _f32(Z)
    lt, t, d = Z.shape[0], Z.shape[1], Z.shape[-1]
    if tuple(gout.shape) != (num_levels + 1, t, t):
        raise ValueError(f"gout must be (num_levels+1, T, T) = {(num_levels + 1, t, t)}")
    gout = _f32(gout)
    if gZ is None:
        gZ = torch.zeros(Z.shape, dtype=torch.float32, device=Z.device)
    nb = lib.gpsig_tens_gram_vjp_workspace_bytes(lt, t, int(increments), d, num_levels, base_kind(base))
    ws = workspace(Z.device, nb) if nb else None
    rc = lib.gpsig_tens_gram_vjp(Z.data_ptr(), lt, t, int(increments), d, num_levels, base_kind(base), gout.data_ptr(),
                                 gZ.data_ptr(), _ptr(ws), ws.numel() if nb else 0, _stream(Z.device))
    L.check(rc, "gpsig_tens_gram_vjp")
    return gZ


EMBEDDINGS = {"linear": 0, "rbf": 1}


def rescaled(Z: torch.Tensor, X: torch.Tensor, num_levels: int, embedding: str = "linear") -> torch.Tensor:
    """VOSF <S(x),(I - Lambda_t) S(x)> per level: Z (LT,T,D), X (N,L,D) -> (M+1, N, T)."""
    _require_cuda(Z, X)
    lib = L.load()
    Z, X = _f32(Z), _f32(X)
    lt, t, d = Z.shape
    n, l, _ = X.shape
    out = torch.empty((num_levels + 1, n, t), dtype=torch.float32, device=X.device)
    ws = workspace(X.device, lib.gpsig_rescaled_workspace_bytes(n, num_levels))
    rc = lib.gpsig_rescaled(Z.data_ptr(), lt, t, X.data_ptr(), n, l, d, num_levels, EMBEDDINGS[embedding],
                            out.data_ptr(), ws.data_ptr(), ws.numel(), _stream(X.device))
    L.check(rc, "gpsig_rescaled")
    return out
