"""Timing of the matrix-core fp32 GEMM (gpsig_amd/csrc/gemm.hip) on the SVGP step's seed shapes: the Kuf
forward seed S = A DX^T (10000 component rows x 24950 increments x 126 channels, NT), the same at H = 1, and
the NN / TN forms of that product.  One JSON line per shape: ms per call and TFLOP/s (2 M N K)."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpsig_amd import _lib as L

SHAPES = [(0, 1, 10000, 24950, 126), (0, 1, 5000, 24950, 126), (0, 0, 10000, 24950, 126),
          (1, 0, 10000, 24950, 126), (0, 1, 4096, 4096, 4096)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    lib = L.load()
    st = torch.cuda.current_stream()
    g = torch.Generator(device="cuda").manual_seed(0)
    for ta, tb, M, N, K in SHAPES:
        A = torch.randn((K, M) if ta else (M, K), device="cuda", generator=g)
        B = torch.randn((N, K) if tb else (K, N), device="cuda", generator=g)
        C = torch.empty((M, N), device="cuda")

        def run():
            L.check(lib.gpsig_gemm_f32(ta, tb, M, N, K, 1.0, A.data_ptr(), A.shape[1], B.data_ptr(), B.shape[1], 0.0,
                                       C.data_ptr(), N, st.cuda_stream), "gpsig_gemm_f32")
        run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            run()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.reps
        ref = (A.T if ta else A)[:64].double() @ (B.T if tb else B).double()
        err = (C[:64].double() - ref).abs().max().item()
        print(json.dumps(dict(op=("T" if ta else "N") + ("T" if tb else "N"), M=M, N=N, K=K, ms=ms,
                              tflops=2.0 * M * N * K / ms / 1e9, max_err=err)), flush=True)
        del A, B, C


if __name__ == "__main__":
    main()
