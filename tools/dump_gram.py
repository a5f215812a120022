"""Dump GPU Gram levels for a golden fixture (debug helper): python tools/dump_gram.py fixture out.npz"""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
import gpsig_amd
g = np.load(sys.argv[1])
X = g["X"]
N, L, D = X.shape
M = int(g["num_levels"])
k = gpsig_amd.SignatureRBF(L * D, D, M)
t = lambda a: torch.as_tensor(a, device="cuda:0")
Kl = k.K(t(X.reshape(N, -1)), return_levels=True).cpu().numpy()
kn = gpsig_amd.SignatureRBF(L * D, D, M, normalization=False)
raw = kn.K(t(X.reshape(N, -1)), return_levels=True).cpu().numpy()
np.savez(sys.argv[2], Kl=Kl, raw=raw)
