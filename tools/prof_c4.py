import sys, os, numpy as np, torch
sys.path.insert(0, os.getcwd())
import gpsig_amd
T, N, L, D, M = 512, 4096, 100, 5, 5
LT = M*(M+1)//2
rng = np.random.default_rng(2)
for incr in (False, True):
    Z = torch.tensor(rng.standard_normal((LT, T, 2, D) if incr else (LT, T, D)), device="cuda", dtype=torch.float32)
    X = torch.tensor(np.cumsum(rng.standard_normal((N, L, D)), 1).reshape(N, -1) / np.sqrt(L*D), device="cuda", dtype=torch.float32)
    k = gpsig_amd.SignatureRBF(L*D, D, M)
    for _ in range(5):
        with torch.no_grad():
            k.K_tens_vs_seq(Z, X, increments=incr)
    torch.cuda.synchronize()
