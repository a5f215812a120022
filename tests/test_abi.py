"""CPU: the C-ABI library loads, exports every symbol include/gpsig_amd.h declares, and validates
arguments without touching a GPU."""
import ctypes
import os
import re

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "gpsig_amd.h")


def header_symbols():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"\b(gpsig_[a-z_]+)\s*\(", txt)))


def test_header_declares_expected_entry_points():
    syms = header_symbols()
    for s in ["gpsig_sig_gram", "gpsig_sig_diag", "gpsig_pde_gram", "gpsig_pde_diag", "gpsig_tens_vs_seq",
              "gpsig_tens_gram", "gpsig_rescaled", "gpsig_sym_assemble", "gpsig_version"]:
        assert s in syms, s


def test_library_exports_every_header_symbol():
    import gpsig_amd._lib as L
    lib = L.load()
    for s in header_symbols():
        assert hasattr(lib, s), s
    assert b"gfx950" in lib.gpsig_version()


def test_python_signatures_cover_header():
    import gpsig_amd._lib as L
    assert set(header_symbols()) <= set(L.SIGNATURES)


def test_argument_validation_without_gpu():
    import gpsig_amd._lib as L
    lib = L.load()
    # null pointers / bad shapes are rejected before any HIP call
    rc = lib.gpsig_sig_gram(None, 4, 10, None, 4, 10, 3, 4, 1, 0, 1, 0, 0, 4, None, None, None, 0.0, 0,
                            None, 0, 4, None, 0, None)
    assert rc == L.GPSIG_EINVAL
    rc = lib.gpsig_pde_gram(None, 4, 10, None, 4, 10, 3, 9, 1, 0, 0, 4, None, 0, 4, None)
    assert rc == L.GPSIG_EINVAL
    assert lib.gpsig_sig_workspace_bytes(10, 20, 10, 20, 5) > 0


def test_library_binary_targets_gfx950():
    import gpsig_amd._lib as L
    data = open(L.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_product_path_refuses_cpu_tensors():
    import torch
    import gpsig_amd
    from gpsig_amd import ops
    X = torch.zeros(2, 5, 3)
    with pytest.raises(gpsig_amd.GpsigError):
        ops.sig_diag(X, 3)


def test_vjp_and_feature_entry_points_validate_arguments():
    """The gradient / signature entry points reject null pointers and bad shapes before any HIP call."""
    import gpsig_amd._lib as L
    lib = L.load()
    assert lib.gpsig_sig_gram_vjp(None, 4, 10, None, 4, 10, 3, 4, 0, 1, 0, 0, 4, None, 0, None, None, None, 0.0,
                                  None, None, None, None, None, None, None, 0, None) == L.GPSIG_EINVAL
    assert lib.gpsig_sig_gram_state(None, 4, 10, None, 4, 10, 3, 4, 0, 0, 0, 4, None, None, None, 0.0, 0, None,
                                    0, 4, None, 0, None, 0, None) == L.GPSIG_EINVAL
    # saved VJP state: (M-1)(l2-1) + M floats per pair; upper triangle for K(X); DIAG has none
    assert lib.gpsig_sig_state_bytes(4, 6, 10, 5, L.PAIRS_RECT) == 4 * 6 * (4 * 9 + 5) * 4
    assert lib.gpsig_sig_state_bytes(6, 6, 10, 5, L.PAIRS_UPPER) == 21 * (4 * 9 + 5) * 4
    assert lib.gpsig_sig_state_bytes(6, 6, 10, 5, L.PAIRS_DIAG) == 0
    assert lib.gpsig_tens_vs_seq_vjp(None, 6, 2, 0, 3, None, 4, 10, 3, 0, 1, None, None, None, None, None, 0,
                                     None) == L.GPSIG_EINVAL
    assert lib.gpsig_tens_vs_seq_state(None, 6, 2, 0, 3, None, 4, 10, 3, 0, None, None, None, 0,
                                       None) == L.GPSIG_EINVAL
    assert lib.gpsig_tens_gram_vjp(None, 6, 2, 0, 3, 3, 0, None, None, None, 0, None) == L.GPSIG_EINVAL
    # the pair-tile + GEMM path past 32 channels: m (LT T^2), kv (4 LT T^2), [Z_h | 1] and G (LT 2 T (d + 1))
    assert lib.gpsig_tens_gram_vjp_workspace_bytes(10, 64, 1, 3, 4, L.BASE_RBF) == 0
    assert lib.gpsig_tens_gram_vjp_workspace_bytes(10, 64, 1, 46, 4, L.BASE_RBF) == \
        (10 * 64 * 64 + 40 * 64 * 64 + 2 * 20 * 64 * 47) * 4
    assert lib.gpsig_pde_vjp(None, 4, 10, None, 4, 10, 3, 0, 1, 0, 0, 4, None, None, None, None, 0,
                             None) == L.GPSIG_EINVAL
    assert lib.gpsig_signature(None, 4, 10, 3, 3, None, None) == L.GPSIG_EINVAL
    assert lib.gpsig_signature_vjp(None, 4, 10, 3, 3, None, None, None) == L.GPSIG_EINVAL
    assert lib.gpsig_signature_channels(5, 3) == 5 + 25 + 125
    # past the 160 KiB of LDS the levels take per-path workspace slabs (256-byte aligned, <= 1 GiB per launch)
    assert lib.gpsig_signature_workspace_bytes(4, 5, 5, 0) == 0 and lib.gpsig_signature_workspace_bytes(4, 5, 5, 1) == 0
    tot = lib.gpsig_signature_channels(6, 6)  # 55 986 coordinates
    assert lib.gpsig_signature_workspace_bytes(4, 6, 6, 0) == 4 * ((tot + 6 + 63) // 64 * 64) * 4
    assert lib.gpsig_signature_workspace_bytes(4, 6, 6, 1) == 4 * ((4 * tot + 12 + 63) // 64 * 64) * 4
    fake = ctypes.c_void_p(256)  # never dereferenced: the workspace check comes before any launch
    assert lib.gpsig_signature(fake, 4, 10, 6, 6, fake, None) == L.GPSIG_EWORKSPACE
    assert lib.gpsig_signature_vjp(fake, 4, 10, 6, 6, fake, fake, None) == L.GPSIG_EWORKSPACE
    # J = 18 fine columns at dyadic 1: W = 2 per lane, U = 9 lanes, 9 + 9 - 1 = 17 coarse steps, a front every
    # 32 / (2 * 2) = 8 steps -> 3 fronts of (W + REP) x 64 floats per pair
    assert lib.gpsig_pde_vjp_workspace_bytes(2, 10, 10, 1) == 2 * 3 * (2 + 2) * 64 * 4
    # J = 1099 > 64 x 16: two column blocks of 1024 (W = 16, H = 2, 36 fronts each) + fp64 boundary columns
    assert lib.gpsig_pde_vjp_workspace_bytes(2, 10, 1100, 0) == 2 * (2 * 36 * 17 * 64 + 2 * 2 * 10) * 4
    # dyadic > 3: the order-3 layout of the grid whose cells are split 2^(dyadic-3) (tile sub-refinement)
    assert lib.gpsig_pde_vjp_workspace_bytes(2, 10, 10, 4) == lib.gpsig_pde_vjp_workspace_bytes(2, 19, 19, 3)
    assert lib.gpsig_pde_vjp_workspace_bytes(2, 10, 10, 7) == lib.gpsig_pde_vjp_workspace_bytes(2, 145, 145, 3)
    assert lib.gpsig_pde_vjp_workspace_bytes(2, 10, 10, 9) == 0


def test_graph_capture_refuses_host_tensors_and_kernel_to():
    """gpsig_amd.graphs.GraphedCall takes device tensors only; kern.to() keeps parameter leaves."""
    import torch
    import gpsig_amd
    from gpsig_amd.graphs import GraphedCall
    with pytest.raises(ValueError):
        GraphedCall(lambda a: a, torch.zeros(2))
    k = gpsig_amd.SignatureRBF(20, 2, 3, lengthscales=[1.0, 2.0])
    k.lengthscales.requires_grad_(True)
    k.to("cpu")
    assert k.lengthscales.is_leaf and k.lengthscales.requires_grad
    assert gpsig_amd.UntruncSignatureKernel(20, 2).to("cpu").num_features == 2


def test_release_workspaces_clears_cache():
    from gpsig_amd import ops
    ops._ws[("x", 0)] = object()
    ops.release_workspaces()
    assert not ops._ws
