"""Row-block sharding of the signature-kernel Gram over the GPUs of one node.

One process per GPU (torch.distributed; backend "nccl" is RCCL on ROCm, over xGMI).  The reference
has no distributed code; this is the north_star's multi-GPU path:

  * symmetric K(X): the N rows are cut into 2P chunks; rank r evaluates the upper-triangle pairs of
    chunks r and 2P-1-r (equal triangle work per rank), each rank holds X in full (N*L*D*4 bytes:
    33.5 MB at N=8192, L=128, D=8) and computes the per-level diagonal redundantly (N pairs, 1/N of
    the Gram work), so the only data-path collective is ONE all_gather_into_tensor of the finished,
    normalised row blocks, after which a gfx950 kernel mirrors the lower triangle
    (gpsig_sym_assemble);
  * cross K(X, X2): the N1 rows are cut into P equal blocks, one all-gather;
  * the PDE Gram (kernels_pde K) shards the same two ways; the inducing-tensor Kuf (K_tens_vs_seq)
    shards its sequences (columns): each rank evaluates and normalises a contiguous block of
    sequences (the normalisation is per sequence, no collective), one all-gather of the blocks.

The compute and assembly steps are injectable so tests can run the partition / gather / assembly
logic on CPU with the gloo backend (tests/test_distributed.py); the product path uses the HIP ops.
"""
from __future__ import annotations

import contextlib
import math

import torch
import torch.distributed as dist

from . import _lib as L
from . import ops


def _world(group=None):
    if not dist.is_available() or not dist.is_initialized():
        return 0, 1
    return dist.get_rank(group), dist.get_world_size(group)


def triangle_chunks(n: int, world: int, align: int = 1):
    """2*world contiguous row chunks [(start, stop)] as equal as possible (boundaries rounded to
    `align`), and B = the largest chunk (every rank ships two B-row slots in the all-gather)."""
    bounds = [min(n, int(round(c * n / (2 * world) / align)) * align) for c in range(2 * world + 1)]
    bounds[-1] = n
    chunks = [(bounds[c], bounds[c + 1]) for c in range(2 * world)]
    B = max(1, max(e - s for s, e in chunks))
    return chunks, B


def rank_chunks(n: int, world: int, rank: int, align: int = 1):
    chunks, B = triangle_chunks(n, world, align)
    return chunks[rank], chunks[2 * world - 1 - rank], B


def row_offsets(n: int, world: int, levels: int, align: int = 1, device=None) -> torch.Tensor:
    """Element offset (level 0) of every global row inside the gathered (world, 2, levels, B, n)
    buffer (rank, chunk slot, level, row-in-chunk, column); the level stride is B*n."""
    chunks, B = triangle_chunks(n, world, align)
    off = torch.empty(n, dtype=torch.int64)
    for c, (s, e) in enumerate(chunks):
        if e <= s:
            continue
        r, slot = (c, 0) if c < world else (2 * world - 1 - c, 1)
        base = ((r * 2 + slot) * levels * B) * n
        off[s:e] = base + (torch.arange(e - s, dtype=torch.int64)) * n
    return off.to(device) if device is not None else off


def _hip_compute(X, levels_out, rows, out, out_row0, **kw):
    return ops.sig_gram(X, None, rows=rows, out=out, out_row0=out_row0, **kw)


def _hip_assemble(gathered, row_off, level_stride, n, levels):
    return ops.sym_assemble(gathered, row_off, level_stride, n, levels)


def sym_local_blocks(X: torch.Tensor, num_levels: int, rank: int, world: int, *, out_mode: int = L.OUT_NORM_SUM,
                     compute=None, **kw) -> torch.Tensor:
    """Rank `rank`'s share of the symmetric Gram: its two row chunks r and 2P-1-r, (2, levels, B, n)
    (chunk slot, level, row, column), rows past a chunk's end zero.  This is exactly the tensor the rank
    contributes to the all-gather."""
    compute = compute or _hip_compute
    n = X.shape[0]
    levels = 1 if out_mode == L.OUT_NORM_SUM else num_levels + 1
    (a0, a1), (b0, b1), B = rank_chunks(n, world, rank)
    # (chunk slot, level, row, col): each chunk's block is contiguous for the kernel's output layout
    local = torch.zeros((2, levels, B, n), dtype=torch.float32, device=X.device)
    if a1 > a0:
        compute(X, levels, (a0, a1), local[0], a0, num_levels=num_levels, out_mode=out_mode, **kw)
    if b1 > b0:
        compute(X, levels, (b0, b1), local[1], b0, num_levels=num_levels, out_mode=out_mode, **kw)
    return local


def sym_from_gathered(gathered: torch.Tensor, n: int, world: int, levels: int, assemble=None) -> torch.Tensor:
    """Full (levels, n, n) symmetric Gram from the all-gathered (world * 2 * levels * B, n) buffer."""
    assemble = assemble or _hip_assemble
    _, B = triangle_chunks(n, world)
    row_off = row_offsets(n, world, levels, device=gathered.device)
    return assemble(gathered, row_off, B * n, n, levels)


def _no_phase(name):
    return contextlib.nullcontext()


def sharded_sym_gram(X: torch.Tensor, num_levels: int, *, out_mode: int = L.OUT_NORM_SUM, group=None,
                     compute=None, assemble=None, phase=None, **kw) -> torch.Tensor:
    """Full symmetric Gram on every rank.  kw: order, base, difference, rs1/rs2, scale, jitter.
    phase(name) -> context manager around the "all_gather" and "assemble" steps (bench.py times them
    with HIP events; the Gram launches are timed through `compute`).

    Returns (n, n) for OUT_NORM_SUM, else (num_levels+1, n, n).
    """
    compute = compute or _hip_compute
    phase = phase or _no_phase
    rank, world = _world(group)
    n = X.shape[0]
    levels = 1 if out_mode == L.OUT_NORM_SUM else num_levels + 1
    if world == 1:
        out = torch.empty((levels, n, n), dtype=torch.float32, device=X.device)
        compute(X, levels, (0, n), out, 0, num_levels=num_levels, out_mode=out_mode, **kw)
        return out[0] if out_mode == L.OUT_NORM_SUM else out
    local = sym_local_blocks(X, num_levels, rank, world, out_mode=out_mode, compute=compute, **kw)
    gathered = torch.empty((world * local.numel() // n, n), dtype=torch.float32, device=X.device)
    with phase("all_gather"):
        dist.all_gather_into_tensor(gathered, local.reshape(-1, n), group=group)
    with phase("assemble"):
        full = sym_from_gathered(gathered, n, world, levels, assemble)
    return full[0] if out_mode == L.OUT_NORM_SUM else full


def cross_local_block(X: torch.Tensor, X2: torch.Tensor, num_levels: int, rank: int, world: int, *,
                      out_mode: int = L.OUT_NORM_SUM, compute=None, **kw) -> torch.Tensor:
    """Rank `rank`'s row block of K(X, X2): (levels, R, n2), R = ceil(n1 / world), rows past n1 zero."""
    n1, n2 = X.shape[0], X2.shape[0]
    levels = 1 if out_mode == L.OUT_NORM_SUM else num_levels + 1
    R = int(math.ceil(n1 / world))
    r0, r1 = min(rank * R, n1), min((rank + 1) * R, n1)
    local = torch.zeros((levels, R, n2), dtype=torch.float32, device=X.device)
    if compute is None:
        if r1 > r0:
            ops.sig_gram(X, X2, num_levels, rows=(r0, r1), out=local, out_row0=r0, out_mode=out_mode, **kw)
    else:
        compute(X, X2, levels, (r0, r1), local, r0, num_levels=num_levels, out_mode=out_mode, **kw)
    return local


def cross_from_gathered(g: torch.Tensor, n1: int) -> torch.Tensor:
    """(levels, n1, n2) from the all-gathered (world, levels, R, n2) row blocks."""
    world, levels, R, n2 = g.shape
    return g.permute(1, 0, 2, 3).reshape(levels, world * R, n2)[:, :n1]


def sharded_cross_gram(X: torch.Tensor, X2: torch.Tensor, num_levels: int, *, out_mode: int = L.OUT_NORM_SUM,
                       group=None, compute=None, **kw) -> torch.Tensor:
    """K(X, X2) row-sharded over ranks; full (n1, n2) [or (levels, n1, n2)] on every rank."""
    rank, world = _world(group)
    n1, n2 = X.shape[0], X2.shape[0]
    local = cross_local_block(X, X2, num_levels, rank, world, out_mode=out_mode, compute=compute, **kw)
    levels, R = local.shape[0], local.shape[1]
    if world == 1:
        full = local
    else:
        g = torch.empty((world, levels, R, n2), dtype=torch.float32, device=X.device)
        dist.all_gather_into_tensor(g.view(world * levels * R, n2), local.reshape(levels * R, n2), group=group)
        full = cross_from_gathered(g, n1)
    return full[0] if out_mode == L.OUT_NORM_SUM else full


def _pde_compute(X, levels_out, rows, out, out_row0, num_levels=None, out_mode=None, dyadic=0, solver=1):
    return ops.pde_gram(X, None, dyadic, solver, rows=rows, out=out[0], out_row0=out_row0)


def sharded_pde_gram(X: torch.Tensor, X2: torch.Tensor | None = None, dyadic: int = 0, solver: int = 1, *,
                     group=None, compute=None, assemble=None) -> torch.Tensor:
    """PDE signature-kernel Gram (gpsig_pde_gram) row-sharded over the process group; (n1, n2) on
    every rank.  compute(X, [X2,] levels, rows, out, out_row0, **kw) is injectable for CPU tests."""
    if X2 is None:
        return sharded_sym_gram(X, 0, out_mode=L.OUT_NORM_SUM, group=group, compute=compute or _pde_compute,
                                assemble=assemble, dyadic=dyadic, solver=solver)

    def cross(Xa, Xb, levels, rows, out, out_row0, num_levels=None, out_mode=None, **kw):
        if rows[1] > rows[0]:
            ops.pde_gram(Xa, Xb, dyadic, solver, rows=rows, out=out[0], out_row0=out_row0)

    return sharded_cross_gram(X, X2, 0, out_mode=L.OUT_NORM_SUM, group=group, compute=compute or cross)


def column_blocks(n: int, world: int):
    """P contiguous blocks of ceil(n / P) sequences; block r = [r*C, min(n, (r+1)*C))."""
    C = int(math.ceil(n / world))
    return [(min(r * C, n), min((r + 1) * C, n)) for r in range(world)], C


def sharded_columns(fn, X: torch.Tensor, group=None) -> torch.Tensor:
    """Evaluate fn on this rank's contiguous block of sequences X[c0:c1] (fn returns (..., c1-c0)),
    all-gather the blocks along the last axis; the full (..., n) result on every rank."""
    rank, world = _world(group)
    n = X.shape[0]
    if world == 1:
        return fn(X)
    blocks, C = column_blocks(n, world)
    c0, c1 = blocks[rank]
    part = fn(X[c0:c1]) if c1 > c0 else None
    lead = part.shape[:-1] if part is not None else None
    # every rank needs the output's leading shape and dtype: take them from a 1-sequence evaluation
    if part is None:
        probe = fn(X[:1])
        lead, dtype = probe.shape[:-1], probe.dtype
    else:
        dtype = part.dtype
    local = torch.zeros((*lead, C), dtype=dtype, device=X.device)
    if part is not None:
        local[..., :c1 - c0] = part
    g = torch.empty((world, *lead, C), dtype=dtype, device=X.device)
    dist.all_gather_into_tensor(g.view(world * local.numel()), local.contiguous().view(-1), group=group)
    full = g.movedim(0, -2).reshape(*lead, world * C)
    return full[..., :n]


def sharded_K_tens_vs_seq(kern, Z, X, return_levels=False, increments=False, group=None):
    """SignatureKernel.K_tens_vs_seq (gpsig/kernels.py:571-620) with the sequences sharded over the
    process group (normalisation is per sequence: no collective besides the all-gather)."""
    Xt = X if isinstance(X, torch.Tensor) else torch.as_tensor(X, device="cuda")
    return sharded_columns(lambda Xb: kern.K_tens_vs_seq(Z, Xb, return_levels=return_levels,
                                                          increments=increments), Xt, group)


def sharded_pde_K(kern, X, X2=None, group=None):
    """UntruncSignatureKernel.K (PDE cross Gram) row-sharded over the process group."""
    Xs = kern._prep(X)
    X2s = None if X2 is None else kern._prep(X2)
    K = sharded_pde_gram(Xs, X2s, kern.order, kern.solver, group=group)
    return (float(kern.sigma) * K).to(kern._dt(X))


def sharded_K(kern, X, X2=None, return_levels=False, group=None):
    """SignatureKernel.K (gpsig/kernels.py:402-477) evaluated row-sharded over the process group."""
    Xs = kern._prep(X)
    scale = kern._scale_vec(Xs.device)
    mode = L.OUT_NORM_LEVELS if return_levels else L.OUT_NORM_SUM
    common = dict(order=kern.order, base=kern.base, difference=kern.difference, scale=scale)
    if X2 is None:
        rs = kern._rsqrt_diag(Xs) if kern.normalization else None
        return sharded_sym_gram(Xs, kern.num_levels, out_mode=mode, group=group, rs1=rs, rs2=rs,
                                jitter=kern.jitter if kern.normalization else 0.0, **common)
    X2s = kern._prep(X2)
    rs1 = rs2 = None
    if kern.normalization:
        rs1, rs2 = kern._rsqrt_diag(Xs), kern._rsqrt_diag(X2s)
    return sharded_cross_gram(Xs, X2s, kern.num_levels, out_mode=mode, group=group, rs1=rs1, rs2=rs2, **common)
