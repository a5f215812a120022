#!/usr/bin/env python
"""Benchmark: signature-kernel Gram entries/s on MI355X (BASELINE.json metric).

One step = one full normalised K(X) of SignatureRBF (reference gpsig/kernels.py:402-477) over the
synthetic workload, inputs resident in HBM: lengthscale scaling, the per-level diagonal (for the
normalisation), the Gram recursion kernel with the fused normalisation / sigma*variances / level-sum
epilogue, and -- at N > 1 GPUs -- the RCCL all-gather of the row blocks plus the gfx950 mirror
assembly, so every rank ends with the full N x N matrix ("scaling": "strong": the total Gram is fixed).

    python bench.py                        # N=1, headline workload
    torchrun --nproc-per-node 8 bench.py --gpus 8

Prints ONE JSON line on rank 0 (contract in the task statement / DESIGN.md "Measurement").
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

WORKLOADS = {
    # north_star target configuration (SURVEY.md 8 "H")
    "H": dict(n=4096, l=128, d=5, m=5),
    # BASELINE.json configs[1]
    "C2": dict(n=1024, l=100, d=5, m=5),
    # BASELINE.json configs[4] (8 GPUs)
    "C5": dict(n=8192, l=128, d=8, m=6),
}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)


def synthetic(n, l, d, seed=0):
    """X = cumsum(N(0,1)) / sqrt(L*D), float32."""
    rng = np.random.default_rng(seed)
    return (np.cumsum(rng.standard_normal((n, l, d)), axis=1) / np.sqrt(l * d)).astype(np.float32)


# ----------------------------------------------------------------------------- CPU baseline
def _cpu_worker(args):
    seconds, n_blk, l, d, m, seed = args
    os.environ["OMP_NUM_THREADS"] = "1"
    os.environ["OPENBLAS_NUM_THREADS"] = "1"
    from oracle import kernels_ref as kr  # checker/baseline only (oracle is test infrastructure)
    k = kr.SignatureKernelRef(l * d, d, m, normalization=False)
    X = synthetic(2 * n_blk, l, d, seed).astype(np.float64)
    t0 = time.perf_counter()
    done = 0
    while True:
        k.K_seq(X[:n_blk], X[n_blk:])
        done += n_blk * n_blk
        if time.perf_counter() - t0 >= seconds:
            break
    return done, time.perf_counter() - t0


def _check_worker(args):
    """Raw per-level Gram blocks (levels, a1-a0, b1-b0) of the float64 oracle for one block pair, and
    the raw per-level diagonal of the rows of block a when it is a diagonal block."""
    Xs, (a0, a1, b0, b1), l, d, m = args
    os.environ["OMP_NUM_THREADS"] = "1"
    from oracle import kernels_ref as kr  # checker only
    k = kr.SignatureKernelRef(l * d, d, m, normalization=False)
    blk = k.K_seq(Xs[a0:a1], Xs[b0:b1])
    diag = k.K_seq_diag(Xs[a0:a1]) if a0 == b0 else None
    return (a0, a1, b0, b1), blk, diag


def oracle_subsample(Xnp, S, l, d, m, jitter, procs, blk=16):
    """SURVEY.md 8d parity sample: the normalised K of the sequences S (the restriction of the normalised
    Gram to S equals K(X[S]) -- normalisation is per sequence), the float64 oracle evaluated in blk x blk
    block pairs (upper triangle) over a process pool, normalised as kernels.py:402-477 with the jitter."""
    Xs = Xnp[S].astype(np.float64)
    ns = len(S)
    jobs = [(Xs, (a, min(a + blk, ns), b, min(b + blk, ns)), l, d, m)
            for a in range(0, ns, blk) for b in range(a, ns, blk)]
    raw = np.zeros((m + 1, ns, ns))
    dg = np.zeros((m + 1, ns))
    with mp.get_context("spawn").Pool(procs) as pool:
        for (a0, a1, b0, b1), blkv, diag in pool.imap_unordered(_check_worker, jobs):
            raw[:, a0:a1, b0:b1] = blkv
            raw[:, b0:b1, a0:a1] = blkv.transpose(0, 2, 1)
            if diag is not None:
                dg[:, a0:a1] = diag
    ds = np.sqrt(dg + jitter)
    K = (raw + jitter * np.eye(ns)[None]) / (ds[:, :, None] * ds[:, None, :])
    return K.sum(0)


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:  # pragma: no cover
        pass
    return "unknown"


def cpu_procs():
    """Every CPU in the affinity mask, capped at the CPU share the job is given (OMP_NUM_THREADS, 16 on
    the GPU boxes, whose affinity mask shows the whole host)."""
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        affinity = os.cpu_count() or 1
    share = int(os.environ.get("OMP_NUM_THREADS", affinity) or affinity)
    return max(1, min(affinity, share)), affinity


def cpu_baseline(l, d, m, seconds=15.0, n_blk=8):
    """The fp64 NumPy restatement of the reference dataflow, one single-threaded process per core."""
    procs, affinity = cpu_procs()
    with mp.get_context("spawn").Pool(procs) as pool:
        res = pool.map(_cpu_worker, [(seconds, n_blk, l, d, m, 100 + i) for i in range(procs)])
    entries = sum(r[0] for r in res)
    wall = max(r[1] for r in res)
    return dict(value=entries / wall, unit="entries/s", cores=procs, affinity_cores=affinity,
                cpu_model=_cpu_model(), kind="port",
                sample=(f"{procs} single-threaded processes (one per core of the job's CPU share; affinity "
                        f"mask {affinity}) x {wall:.1f}s of {n_blk}x{n_blk}-pair raw per-level Gram blocks, "
                        f"L={l}, D={d}, M={m}: oracle/kernels_ref.py float64 NumPy restatement of the "
                        f"reference dataflow (materialised base-kernel tensor, exclusive cumsums)"))


# ----------------------------------------------------------------------------- main
def hbm_copy_probe(dev, nbytes=1 << 30, reps=20):
    """Achievable HBM bandwidth (GB/s): read + write bytes of a 1 GiB device-to-device copy, timed with
    events after the measured steps (outside the timed region)."""
    import torch
    a = torch.empty(nbytes // 4, dtype=torch.float32, device=dev).fill_(1.0)
    b = torch.empty_like(a)
    for _ in range(3):
        b.copy_(a)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        b.copy_(a)
    e1.record()
    e1.synchronize()
    gbs = 2.0 * nbytes * reps / (e0.elapsed_time(e1) / 1e3) / 1e9
    del a, b
    return gbs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="H", choices=sorted(WORKLOADS))
    ap.add_argument("--nseq", "--n", dest="n", type=int, help="override the workload N")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-check", action="store_true")
    ap.add_argument("--no-probe", action="store_true", help="skip the HBM copy-bandwidth probe")
    ap.add_argument("--seed-engine", default="valu", choices=["valu", "mfma"],
                    help="RBF seed dots on packed VALU FMAs (default) or on the matrix cores (A/B arm)")
    ap.add_argument("--gram-path", default="fused", choices=["fused", "split"],
                    help="fused Gram kernel (default) or the split diagnostic of SURVEY.md 8d: a producer "
                         "launch writes the cells dM to HBM, a consumer streams them through the recursion")
    ap.add_argument("--backend", default="nccl",
                    help="process-group backend (nccl = RCCL; gloo only to rehearse N>1 ranks on one GPU)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "r6_gram_counters.json"),
                    help="per-launch HBM bytes of the Gram kernel from a PMC pass (profiles/*.json)")
    ap.add_argument("--check-rows", type=int, default=256,
                    help="rows of the max_abs_err subsample (SURVEY.md 8d: 256 for large N)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} (launch N > 1 with "
                         f"torch.distributed.run --nproc-per-node N)")
    dev = torch.device("cuda", local_rank % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.backend)
        assert dist.get_world_size() == args.gpus, (dist.get_world_size(), args.gpus)

    import gpsig_amd
    from gpsig_amd import _lib as L
    from gpsig_amd import distributed as gdist
    from gpsig_amd import ops

    wl = dict(WORKLOADS[args.workload])
    if args.n:
        wl["n"] = args.n
    n, l, d, m = wl["n"], wl["l"], wl["d"], wl["m"]
    Xnp = synthetic(n, l, d)
    X = torch.as_tensor(Xnp.reshape(n, l * d), device=dev)
    kern = gpsig_amd.SignatureRBF(l * d, d, m)

    # events around every launch of the dominant kernel (the Gram recursion), on its stream
    ev = []
    rows_done = [0]

    def timed_compute(Xs, levels_out, rows, out, out_row0, **kw):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        r = ops.sig_gram(Xs, None, rows=rows, out=out, out_row0=out_row0, **kw)
        e1.record()
        ev.append((e0, e1))
        # pairs the launch evaluates: symmetric K(X) computes b >= a only (the mirror is a store)
        a0, a1 = rows
        rows_done[0] += (a1 - a0) * n - (a1 * (a1 - 1) - a0 * (a0 - 1)) // 2
        return r

    # HIP events around the collective and the mirror assembly (N > 1), on the current stream
    phases = {"all_gather": [], "assemble": []}

    class phase:
        def __init__(self, name):
            self.name = name

        def __enter__(self):
            self.e0 = torch.cuda.Event(enable_timing=True)
            self.e0.record()

        def __exit__(self, *exc):
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            phases[self.name].append((self.e0, e1))

    gram_base = (L.BASE_RBF | (L.BASE_SEED_MFMA if args.seed_engine == "mfma" else 0)
                 | (L.GRAM_SPLIT if args.gram_path == "split" else 0))

    def step():
        Xs = kern._prep(X)
        rs = kern._rsqrt_diag(Xs)
        return gdist.sharded_sym_gram(Xs, m, out_mode=L.OUT_NORM_SUM, compute=timed_compute, rs1=rs, rs2=rs,
                                      scale=kern._scale_vec(dev), jitter=kern.jitter, order=kern.order,
                                      base=gram_base, difference=kern.difference, phase=phase)

    for _ in range(args.warmup):
        K = step()
    torch.cuda.synchronize()
    ev.clear()
    for v in phases.values():
        v.clear()
    rows_done[0] = 0
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        K = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # dominant-kernel roofline: algorithmic bytes per Gram entry
    kern_ms = sum(a.elapsed_time(b) for a, b in ev)
    launches = len(ev)
    entries_per_launch = rows_done[0] / max(launches, 1)  # evaluated (upper-triangle) pairs
    b_entry = 4 * (l - 1) * (l - 1) + 4 * (m + 1)
    avg_launch_s = kern_ms / 1e3 / max(launches, 1)
    achieved = entries_per_launch * b_entry / avg_launch_s / 1e9
    traffic, prof = None, {}
    # the committed profile is of the default single-GPU launch; other runs report traffic null
    if (args.traffic_json and os.path.exists(args.traffic_json) and args.workload == "H" and not args.n
            and args.seed_engine == "valu" and args.gram_path == "fused" and world == 1):
        with open(args.traffic_json) as f:
            prof = json.load(f)
        traffic = prof.get("hbm_bytes_per_launch")

    probe = hbm_copy_probe(dev) if rank == 0 and not args.no_probe else None
    value = args.steps * n * n / elapsed
    out = {
        "metric": "sig-kernel Gram entries/sec (N, len L, dim D, level M); max-abs err vs ref",
        "value": value,
        "unit": "entries/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic random walks X = cumsum(N(0,1))/sqrt(L*D), seed 0 (SURVEY.md 8d)",
        "config": {"workload": f"SignatureRBF K(X) normalised, N={n}, L={l}, D={d}, M={m}, order=1",
                   "global_batch": n, "seq_len": l, "parallelism": f"row-shard{world}" if world > 1 else "single"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     # frac is an effective-bandwidth ratio (SURVEY.md 8d's algorithmic bytes of the
                     # materialised-tile design / HBM peak); the fused kernel's physical limiter is VALU
                     # issue, whose busy fraction from the PMC profile is valu_busy below
                     "frac_kind": "effective-bandwidth (algorithmic bytes / HBM peak)",
                     "kernel": "sig_fo_kernel", "seed_engine": args.seed_engine, "gram_path": args.gram_path,
                     "launch_ms": avg_launch_s * 1e3, "bytes_per_entry": b_entry,
                     "entries_per_launch": entries_per_launch,
                     # the fused kernel never materialises the tile: physically it is VALU-issue bound
                     "physical_bound": "valu", "valu_busy": prof.get("valu_busy"),
                     "profile": os.path.relpath(args.traffic_json, ROOT) if prof else None,
                     # the datasheet peak and a measured device-to-device copy (read + write
                     # GB/s).  No fraction against the probe: `achieved` is an effective bandwidth of
                     # algorithmic bytes the fused kernel never moves, so a ratio to a copy is meaningless.
                     "peak_probe": probe},
    }
    # per-rank breakdown of a step (ms): the Gram launches, the all-gather and the mirror assembly
    per_step = lambda evs: sum(a.elapsed_time(b) for a, b in evs) / args.steps  # noqa: E731
    mine = {"rank": rank, "gram_ms": per_step(ev), "gram_launches": len(ev) // max(args.steps, 1),
            "all_gather_ms": per_step(phases["all_gather"]), "assemble_ms": per_step(phases["assemble"]),
            "step_ms": elapsed / args.steps * 1e3}
    if world > 1:
        ranks = [None] * world
        dist.all_gather_object(ranks, mine)
        backend = dist.get_backend()
        lib = None
        if backend == "nccl":
            v = torch.cuda.nccl.version()
            lib = "RCCL " + (".".join(map(str, v)) if isinstance(v, tuple) else str(v))
        out["distributed"] = {"backend": backend, "collective_library": lib, "world_size": world,
                              "per_rank": ranks,
                              # all_gather_into_tensor output: world x 2 chunk slots x B rows x N fp32
                              "gathered_bytes": world * 2 * gdist.triangle_chunks(n, world)[1] * n * 4}
    else:
        out["breakdown"] = mine
    if rank == 0 and not args.no_check:
        # parity on a bounded subsample (256 rows): the normalised Gram restricted to a subset
        # S of the sequences equals K(X[S]) (per-sequence diagonals), evaluated by the float64 oracle
        S = np.unique(np.linspace(0, n - 1, min(n, args.check_rows)).astype(int))
        Kref = oracle_subsample(Xnp, S, l, d, m, kern.jitter, cpu_procs()[0])
        Si = torch.as_tensor(S, device=dev)
        got = K[Si][:, Si].double().cpu().numpy()
        out["max_abs_err"] = float(np.abs(got - Kref).max())
        out["max_abs_ref"] = float(np.abs(Kref).max())
        out["check_rows"] = len(S)
    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(l, d, m, seconds=args.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
