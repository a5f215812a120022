"""Diagnostic: closed-form scaling contraction (autograd._scaling_contraction) on the GPU vs fp64 CPU
autodiff of the reference graph, at the test_ho_grad_gpu shapes (unnormalised, cross, per level)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np, torch
from conftest import golden
from oracle import autodiff_ref as ar
import gpsig_amd
from gpsig_amd import autograd as ag, ops
g = golden("linear_chen.npz"); X = g["X"]; N, L, D = X.shape; M = int(g["num_levels"])
X2 = np.cumsum(np.random.default_rng(3).standard_normal((7, L, D)), 1) / np.sqrt(L * D)
G = np.random.default_rng(4).standard_normal((M + 1, N, 7))
ls = np.array([0.7, 1.3, 1.0]); var = np.linspace(0.5, 1.5, M + 1)
xs = torch.tensor(X / ls, requires_grad=True); x2s = torch.tensor(X2 / ls, requires_grad=True)
Kq = ar.K(xs, x2s, M, base="linear", normalization=False, scale=torch.tensor(var), order=M, return_levels=True)
(Kq * torch.tensor(G)).sum().backward()
e_ref = ((xs.detach() * xs.grad).sum((0, 1)) + (x2s.detach() * x2s.grad).sum((0, 1))).numpy()
Xd, X2d = xs.detach().cuda(), x2s.detach().cuda()
S = ops.signature(Xd, M).double().cpu()
Sr = torch.stack([ar.signature(s, M) for s in xs.detach()])
print("sig rel", ((S - Sr).norm() / Sr.norm()).item())
gK = torch.tensor(G, device="cuda") * torch.tensor(var, device="cuda")[:, None, None]
e = ag._scaling_contraction(Xd, X2d, M, gK).cpu().numpy()
print("e_ref", e_ref, "e", e, "rel", np.linalg.norm(e - e_ref) / np.linalg.norm(e_ref))
k = gpsig_amd.SignatureLinear(L * D, D, M, order=M, normalization=False)
k.lengthscales = torch.tensor(ls, device="cuda", requires_grad=True)
k.variances = torch.tensor(var, device="cuda", requires_grad=True)
Xt = torch.tensor(X.reshape(N, -1), device="cuda", requires_grad=True)
X2t = torch.tensor(X2.reshape(7, -1), device="cuda", requires_grad=True)
K = k.K(Xt, X2t, return_levels=True)
print("K dtype", K.dtype)
(K * torch.as_tensor(G, device="cuda")).sum().backward()
gl = k.lengthscales.grad.cpu().numpy()
print("gl", gl, "ref", -e_ref / ls, "rel", np.linalg.norm(gl + e_ref / ls) / np.linalg.norm(e_ref / ls))
print("closed form", ag._scaling_closed_form(k._cfg(True), Xd, X2d), k._cfg(True))
