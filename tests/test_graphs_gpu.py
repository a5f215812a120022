"""hipGraph capture of kernel evaluations (gpsig_amd/graphs.py): a captured K(X) / K(X, X2) /
PDE Kdiag replayed on new inputs equals the eager call and the fp64 oracle."""
import numpy as np
import pytest
import torch

from oracle import kernels_ref as kr

pytestmark = pytest.mark.gpu
DEV = "cuda"


def walks(n, l, d, seed):
    rng = np.random.default_rng(seed)
    return np.cumsum(rng.standard_normal((n, l, d)), axis=1) / np.sqrt(l * d)


def test_graphed_gram_replays_new_inputs():
    import gpsig_amd
    from gpsig_amd.graphs import GraphedCall
    N, L, D, M = 64, 50, 3, 4  # the reference's C1 configuration
    k = gpsig_amd.SignatureRBF(L * D, D, M).to(DEV)
    X0 = torch.tensor(walks(N, L, D, 0).reshape(N, -1), device=DEV, dtype=torch.float32)
    g = GraphedCall(lambda X: k.K(X), X0)
    for seed in (1, 2):
        Xn = walks(N, L, D, seed)
        Xt = torch.tensor(Xn.reshape(N, -1), device=DEV, dtype=torch.float32)
        got = g(Xt).clone()
        with torch.no_grad():
            eager = k.K(Xt)
        assert torch.equal(got, eager)
        ref = kr.SignatureKernelRef(L * D, D, M).K(Xn.reshape(N, -1))
        assert np.abs(got.double().cpu().numpy() - ref).max() <= 1e-5 * np.abs(ref).max()


def test_graphed_cross_gram_and_pde():
    import gpsig_amd
    from gpsig_amd.graphs import GraphedCall
    N1, N2, L, D, M = 16, 24, 30, 4, 5
    k = gpsig_amd.SignatureLinear(L * D, D, M).to(DEV)
    X = torch.tensor(walks(N1, L, D, 3).reshape(N1, -1), device=DEV, dtype=torch.float32)
    Y = torch.tensor(walks(N2, L, D, 4).reshape(N2, -1), device=DEV, dtype=torch.float32)
    g = GraphedCall(lambda a, b: k.K(a, b, return_levels=True), X, Y)
    Y2 = torch.tensor(walks(N2, L, D, 5).reshape(N2, -1), device=DEV, dtype=torch.float32)
    with torch.no_grad():
        assert torch.equal(g(X, Y2).clone(), k.K(X, Y2, return_levels=True))
    kp = gpsig_amd.UntruncSignatureKernel(L * D, D, order=1).to(DEV)
    gp = GraphedCall(lambda a: kp.Kdiag(a), X)
    X2 = torch.tensor(walks(N1, L, D, 6).reshape(N1, -1), device=DEV, dtype=torch.float32)
    with torch.no_grad():
        assert torch.equal(gp(X2).clone(), kp.Kdiag(X2))


def test_graphed_call_rejects_shape_change():
    import gpsig_amd
    from gpsig_amd.graphs import GraphedCall
    k = gpsig_amd.SignatureRBF(20, 2, 3).to(DEV)
    X = torch.zeros(4, 20, device=DEV)
    g = GraphedCall(lambda a: k.K(a), X)
    with pytest.raises(ValueError):
        g(torch.zeros(5, 20, device=DEV))


def test_graph_survives_workspace_release():
    """The captured launches keep addressing valid scratch after ops.release_workspaces()."""
    import gpsig_amd
    from gpsig_amd import ops
    from gpsig_amd.graphs import GraphedCall
    N, L, D, M = 32, 40, 3, 4
    k = gpsig_amd.SignatureRBF(L * D, D, M).to(DEV)
    X0 = torch.tensor(walks(N, L, D, 7).reshape(N, -1), device=DEV, dtype=torch.float32)
    g = GraphedCall(lambda X: k.K(X), X0)
    ops.release_workspaces()
    # allocate on the capture stream: the caching allocator would hand these blocks out first if the
    # graph's scratch had really been freed
    with torch.cuda.stream(g.stream):
        junk = [torch.full((1 << s,), 7.0, device=DEV) for s in range(12, 22) for _ in range(2)]
    torch.cuda.current_stream().wait_stream(g.stream)
    X1 = torch.tensor(walks(N, L, D, 8).reshape(N, -1), device=DEV, dtype=torch.float32)
    got = g(X1).clone()
    torch.cuda.synchronize()
    with torch.no_grad():
        assert torch.equal(got, k.K(X1))
    assert all(bool((j == 7.0).all()) for j in junk)  # the replay wrote only into its own scratch
    del junk
