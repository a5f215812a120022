"""CPU, world_size 2 (gloo): the row-sharding partition, the all-gather layout and the symmetric
assembly of gpsig_amd.distributed reproduce the single-process Gram.  The per-rank compute is the
float64 oracle (stand-in for the GPU kernel, which needs a GPU) and the assembly is a torch
restatement of gpsig_sym_assemble; the GPU kernel itself is covered in test_gram_gpu.py."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from gpsig_amd import distributed as D
from gpsig_amd import _lib as L
from oracle import kernels_ref as kr


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _oracle_levels(X, M):
    k = kr.SignatureKernelRef(X.shape[1] * X.shape[2], X.shape[2], M, normalization=False)
    return torch.as_tensor(k.K_seq(X.numpy().astype(np.float64)), dtype=torch.float32)


def _compute_sym(X, levels, rows, out, out_row0, num_levels, out_mode, full=None, **kw):
    """UPPER-mode semantics of gpsig_sig_gram: rows [r0,r1), pairs b >= a, mirrored inside the window."""
    r0, r1 = rows
    n = X.shape[0]
    for a in range(r0, r1):
        for b in range(a, n):
            v = full[:, a, b] if out_mode != L.OUT_NORM_SUM else full[:, a, b].sum(0, keepdim=True)
            out[:, a - out_row0, b] = v
            if out_row0 <= b < out_row0 + out.shape[1]:
                out[:, b - out_row0, a] = v


def _assemble_torch(gathered, row_off, level_stride, n, levels):
    flat = gathered.reshape(-1)
    out = torch.empty((levels, n, n))
    for l in range(levels):
        for a in range(n):
            for b in range(n):
                r, c = (a, b) if b >= a else (b, a)
                out[l, a, b] = flat[row_off[r] + l * level_stride + c]
    return out


def _worker(rank, world, port, n, M, mode, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(0)
    X = torch.as_tensor(np.cumsum(rng.standard_normal((n, 12, 2)), 1) * 0.2, dtype=torch.float32)
    full = _oracle_levels(X, M)
    seen = []

    class phase:  # bench.py's per-step breakdown hooks (HIP events there)
        def __init__(self, name):
            seen.append(name)

        def __enter__(self):
            return self

        def __exit__(self, *exc):
            return False

    res = D.sharded_sym_gram(X, M, out_mode=mode, compute=lambda *a, **k: _compute_sym(*a, full=full, **k),
                             assemble=_assemble_torch, phase=phase)
    assert seen == ["all_gather", "assemble"], seen
    q.put((rank, res.numpy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("n", [13, 24])
@pytest.mark.parametrize("mode", [L.OUT_NORM_SUM, L.OUT_NORM_LEVELS])
def test_sharded_symmetric_gram_world2(n, mode):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    M = 3
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n, M, mode, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    rng = np.random.default_rng(0)
    X = torch.as_tensor(np.cumsum(rng.standard_normal((n, 12, 2)), 1) * 0.2, dtype=torch.float32)
    full = _oracle_levels(X, M).numpy()
    exp = full.sum(0) if mode == L.OUT_NORM_SUM else full
    for r in (0, 1):
        np.testing.assert_allclose(res[r], exp, rtol=1e-6, atol=1e-7)


def test_triangle_partition_balanced():
    for n, world in [(4096, 8), (4096, 2), (8192, 8), (100, 4)]:
        chunks, B = D.triangle_chunks(n, world)
        covered = sorted(r for s, e in chunks for r in range(s, e))
        assert covered == list(range(n))
        work = []
        for rank in range(world):
            (a0, a1), (b0, b1), _ = D.rank_chunks(n, world, rank)
            work.append(sum(n - a for a in range(a0, a1)) + sum(n - a for a in range(b0, b1)))
        assert max(work) / (sum(work) / world) < 1.06, work


def test_row_offsets_layout():
    n, world, levels = 50, 4, 3
    chunks, B = D.triangle_chunks(n, world)
    off = D.row_offsets(n, world, levels)
    # every row maps to a distinct B*n-aligned slot inside (world, 2, levels, B, n)
    slots = sorted(int(o) // n for o in off)
    assert len(set(slots)) == n and max(off) < world * 2 * levels * B * n


def _run_world2(target, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, 2, port, q) + args) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    return res


def _pde_worker(rank, world, port, q, n, cross):
    from oracle import pde
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(1)
    X = torch.as_tensor(np.cumsum(rng.standard_normal((n, 9, 2)), 1) * 0.3, dtype=torch.float32)
    if cross:
        X2 = X[:5] * 0.7

        def comp(Xa, Xb, levels, rows, out, out_row0, **kw):
            r0, r1 = rows
            if r1 > r0:
                out[0, r0 - out_row0:r1 - out_row0] = torch.as_tensor(
                    pde.pde_gram(Xa[r0:r1].double().numpy(), Xb.double().numpy(), 1, 1), dtype=torch.float32)

        res = D.sharded_pde_gram(X, X2, 1, 1, compute=comp)
    else:
        full = torch.as_tensor(pde.pde_gram(X.double().numpy(), None, 1, 1), dtype=torch.float32)[None]
        res = D.sharded_pde_gram(X, None, 1, 1, compute=lambda *a, **k: _compute_sym(*a, full=full, **k),
                                 assemble=_assemble_torch)
    q.put((rank, res.numpy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("cross", [False, True])
def test_sharded_pde_gram_world2(cross):
    from oracle import pde
    n = 11
    res = _run_world2(_pde_worker, n, cross)
    rng = np.random.default_rng(1)
    X = np.cumsum(rng.standard_normal((n, 9, 2)), 1) * 0.3
    X = X.astype(np.float32).astype(np.float64)
    exp = pde.pde_gram(X, (X[:5] * 0.7).astype(np.float32).astype(np.float64) if cross else None, 1, 1)
    for r in (0, 1):
        np.testing.assert_allclose(res[r], exp, rtol=1e-5, atol=1e-6)


def _cols_worker(rank, world, port, q, n):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    X = torch.arange(n * 3, dtype=torch.float32).reshape(n, 3)
    fn = lambda Xb: torch.stack([Xb.sum(1), Xb[:, 0] * 2.0], 0)[None]  # (1, 2, nb) per block  # noqa: E731
    q.put((rank, D.sharded_columns(fn, X).numpy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("n", [1, 7, 10])
def test_sharded_columns_world2(n):
    res = _run_world2(_cols_worker, n)
    X = torch.arange(n * 3, dtype=torch.float32).reshape(n, 3)
    exp = torch.stack([X.sum(1), X[:, 0] * 2.0], 0)[None].numpy()
    for r in (0, 1):
        np.testing.assert_allclose(res[r], exp)


def test_bench_refuses_world_mismatch():
    """bench.py --gpus N must run as N ranks (torch.distributed.run): a bare launch with --gpus 2 stops
    before touching a device."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2"], capture_output=True,
                       text=True, env=env, timeout=300)
    assert r.returncode != 0 and "WORLD_SIZE=1" in r.stderr, r.stderr[-2000:]


@pytest.mark.gpu
def test_bench_world2_gloo_breakdown(tmp_path):
    """The N-GPU bench line explains itself: a world-2 gloo rehearsal on one GPU reports the backend and
    every rank's Gram / all-gather / assembly ms."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(root, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--nseq", "256", "--backend", "gloo", "--no-cpu",
           "--no-probe", "--check-rows", "32"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")][-1]
    out = json.loads(line)
    assert out["n_gpus"] == 2 and out["max_abs_err"] < 1e-5
    dd = out["distributed"]
    assert dd["backend"] == "gloo" and dd["world_size"] == 2
    assert [p["rank"] for p in dd["per_rank"]] == [0, 1]
    for p in dd["per_rank"]:
        assert p["gram_ms"] > 0 and p["all_gather_ms"] > 0 and p["assemble_ms"] > 0 and p["gram_launches"] == 2
