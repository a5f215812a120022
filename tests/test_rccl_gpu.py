"""GPU: the multi-GPU data path over a real RCCL process group (torch.distributed backend "nccl" = RCCL on ROCm).

One GPU allows a world of one rank only, so the sharded entry points would take their world-1 shortcut; this
test runs the world > 1 code path's own calls -- sym_local_blocks / cross_local_block for every rank share,
dist.all_gather_into_tensor on the RCCL group, sym_from_gathered / cross_from_gathered -- in a child process
that initialises the "nccl" group at world size 1 exactly as bench.py does at N > 1 (device_id, 127.0.0.1
rendezvous), and checks the assembled Gram bitwise against the single-launch one."""
import os
import subprocess
import sys
import textwrap

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

CHILD = textwrap.dedent(r'''
    import os, sys
    import numpy as np
    import torch
    import torch.distributed as dist
    sys.path.insert(0, os.environ["GPSIG_ROOT"])
    import gpsig_amd
    from gpsig_amd import _lib as L
    from gpsig_amd import distributed as D
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev, init_method="tcp://127.0.0.1:" + os.environ["PORT"], rank=0,
                            world_size=1)
    assert dist.get_backend() == "nccl"
    rng = np.random.default_rng(0)
    N, Ln, Dm, M = 37, 24, 3, 4
    X = torch.tensor(np.cumsum(rng.standard_normal((N, Ln, Dm)), 1).reshape(N, -1) / np.sqrt(Ln * Dm), device=dev)
    X2 = torch.tensor(np.cumsum(rng.standard_normal((11, Ln, Dm)), 1).reshape(11, -1) / np.sqrt(Ln * Dm), device=dev)
    k = gpsig_amd.SignatureRBF(Ln * Dm, Dm, M)
    Xs, X2s = k._prep(X), k._prep(X2)
    rs, rs2 = k._rsqrt_diag(Xs), k._rsqrt_diag(X2s)
    kw = dict(rs1=rs, rs2=rs, scale=k._scale_vec(dev), jitter=k.jitter, order=1, base="rbf", difference=True)
    full = D.sharded_sym_gram(Xs, M, out_mode=L.OUT_NORM_SUM, **kw)
    for world in (1, 2, 8):  # the shares of a world-P job, gathered over the RCCL group one share at a time
        parts = []
        for r in range(world):
            local = D.sym_local_blocks(Xs, M, r, world, out_mode=L.OUT_NORM_SUM, **kw)
            g = torch.empty_like(local.reshape(-1, N))
            dist.all_gather_into_tensor(g, local.reshape(-1, N))
            parts.append(g)
        got = D.sym_from_gathered(torch.cat(parts, 0), N, world, 1)
        assert torch.equal(got.reshape(full.shape), full), world
    kwc = dict(rs1=rs, rs2=rs2, scale=k._scale_vec(dev), jitter=k.jitter, order=1, base="rbf", difference=True)
    fullc = D.sharded_cross_gram(Xs, X2s, M, out_mode=L.OUT_NORM_SUM, **kwc)
    blocks = []
    for r in range(4):
        local = D.cross_local_block(Xs, X2s, M, r, 4, out_mode=L.OUT_NORM_SUM, **kwc)
        g = torch.empty_like(local.reshape(-1, local.shape[-1]))
        dist.all_gather_into_tensor(g, local.reshape(-1, local.shape[-1]))
        blocks.append(g.reshape(local.shape))
    gotc = D.cross_from_gathered(torch.stack(blocks), N)
    assert torch.equal(gotc.reshape(fullc.shape), fullc)
    dist.barrier()
    dist.destroy_process_group()
    print("rccl ok", torch.cuda.nccl.version() if hasattr(torch.cuda, "nccl") else "")
''')


def test_rccl_group_gathers_the_sharded_gram_bitwise():
    env = dict(os.environ, GPSIG_ROOT=ROOT, PORT=str(29500 + os.getpid() % 1000))
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "rccl ok" in r.stdout
