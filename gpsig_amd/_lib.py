"""Loader for the gfx950 C-ABI library (include/gpsig_amd.h) via ctypes.

The library is built in-tree (gpsig_amd/libgpsig_amd.so, see gpsig_amd/csrc/Makefile and
__graft_entry__.build()).  ``torch`` is imported first so the library binds to the HIP runtime
torch already loaded (both carry SONAME libamdhip64.so.7): device pointers and the hipStream_t
handed over from torch are then valid in the library.

There is deliberately no fallback: if the shared object is missing or does not export the
expected symbols, every product entry point raises.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GPSIG_AMD_LIB", os.path.join(_HERE, "libgpsig_amd.so"))

GPSIG_OK = 0
GPSIG_EINVAL = -1
GPSIG_EUNSUPPORTED = -2
GPSIG_ELAUNCH = -3
GPSIG_EWORKSPACE = -4
_ERRORS = {
    GPSIG_EINVAL: "invalid argument",
    GPSIG_EUNSUPPORTED: "configuration not supported by the compiled kernels",
    GPSIG_ELAUNCH: "HIP kernel launch failed",
    GPSIG_EWORKSPACE: "workspace too small",
}

BASE_RBF = 0
BASE_LINEAR = 1
BASE_SEED_MFMA = 0x100  # flag: RBF seed dots on the matrix cores (A/B arm, include/gpsig_amd.h)
GRAM_SPLIT = 0x200  # flag: split producer/consumer diagnostic of the first-order Gram (include/gpsig_amd.h)
PAIRS_RECT, PAIRS_UPPER, PAIRS_DIAG = 0, 1, 2
OUT_LEVELS, OUT_NORM_LEVELS, OUT_NORM_SUM, OUT_RSQRT = 0, 1, 2, 3

_P = ctypes.c_void_p
_I = ctypes.c_int
_F = ctypes.c_float
_SZ = ctypes.c_size_t

SIGNATURES = {
    "gpsig_sig_workspace_bytes": (_SZ, [_I, _I, _I, _I, _I]),
    "gpsig_sig_workspace_bytes_ex": (_SZ, [_I, _I, _I, _I, _I, _I, _I]),
    "gpsig_sig_split_bytes": (_SZ, [_I, _I, _I, _I]),
    "gpsig_sig_vjp_workspace_bytes": (_SZ, [_I, _I, _I, _I, _I, _I, _I]),
    "gpsig_sig_gram": (_I, [_P, _I, _I, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I,
                            _P, _P, _P, _F, _I, _P, _I, _I, _P, _SZ, _P]),
    "gpsig_sig_diag": (_I, [_P, _I, _I, _I, _I, _I, _I, _I, _F, _I, _P, _P, _SZ, _P]),
    "gpsig_sig_gram_vjp": (_I, [_P, _I, _I, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P, _I,
                                _P, _P, _P, _F, _P, _P, _P, _P, _P, _P, _P, _SZ, _P]),
    "gpsig_sig_vjp_ho_workspace_bytes": (_SZ, [_I, _I, _I, _I, _I, _I, _I, _I]),
    "gpsig_sig_gram_vjp_ho": (_I, [_P, _I, _I, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P, _I,
                                   _P, _P, _P, _F, _P, _P, _P, _P, _P, _P, _SZ, _P]),
    "gpsig_sig_state_bytes": (_SZ, [_I, _I, _I, _I, _I]),
    "gpsig_sig_gram_state": (_I, [_P, _I, _I, _P, _I, _I, _I, _I, _I, _I, _I, _I, _P, _P, _P, _F, _I, _P,
                                  _I, _I, _P, _SZ, _P, _SZ, _P]),
    "gpsig_pde_gram": (_I, [_P, _I, _I, _P, _I, _I, _I, _I, _I, _I, _I, _I, _P, _I, _I, _P]),
    "gpsig_pde_diag": (_I, [_P, _I, _I, _I, _I, _I, _P, _P]),
    "gpsig_pde_vjp_workspace_bytes": (_SZ, [_I, _I, _I, _I]),
    "gpsig_pde_vjp": (_I, [_P, _I, _I, _P, _I, _I, _I, _I, _I, _I, _I, _I, _P, _P, _P, _P, _SZ, _P]),
    "gpsig_pde_fronts": (_I, [_P, _I, _I, _P, _I, _I, _I, _I, _I, _I, _I, _I, _P, _P, _SZ, _P]),
    "gpsig_pde_vjp_fronts": (_I, [_P, _I, _I, _P, _I, _I, _I, _I, _I, _I, _I, _I, _P, _P, _P, _P, _SZ, _P]),
    "gpsig_sym_assemble": (_I, [_P, _P, ctypes.c_longlong, _I, _I, _P, _P]),
    "gpsig_pde_scratch_bytes": (_SZ, [_I, _I, _I, _I, _I, _I, _I]),
    "gpsig_pde_gram_ex": (_I, [_P, _I, _I, _P, _I, _I, _I, _I, _I, _I, _I, _I, _P, _I, _I, _P, _SZ, _P]),
    "gpsig_pde_diag_ex": (_I, [_P, _I, _I, _I, _I, _I, _P, _P, _SZ, _P]),
    "gpsig_pde_vjp_scratch_bytes": (_SZ, [_I, _I, _I, _I, _I, _I, _I]),
    "gpsig_pde_vjp_ex": (_I, [_P, _I, _I, _P, _I, _I, _I, _I, _I, _I, _I, _I, _P, _P, _P, _P, _SZ, _P, _SZ, _P]),
    "gpsig_pde_fronts_ex": (_I, [_P, _I, _I, _P, _I, _I, _I, _I, _I, _I, _I, _I, _P, _P, _SZ, _P, _SZ, _P]),
    "gpsig_pde_vjp_fronts_ex": (_I, [_P, _I, _I, _P, _I, _I, _I, _I, _I, _I, _I, _I, _P, _P, _P, _P, _SZ, _P, _SZ,
                                     _P]),
    "gpsig_tens_vs_seq": (_I, [_P, _I, _I, _I, _I, _P, _I, _I, _I, _I, _I, _I, _P, _P, _SZ, _P]),
    "gpsig_tens_gram_workspace_bytes": (_SZ, [_I, _I, _I]),
    "gpsig_tens_gram": (_I, [_P, _I, _I, _I, _I, _I, _I, _P, _P, _SZ, _P]),
    "gpsig_tens_vs_seq_vjp": (_I, [_P, _I, _I, _I, _I, _P, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _SZ, _P]),
    "gpsig_tens_vs_seq_state": (_I, [_P, _I, _I, _I, _I, _P, _I, _I, _I, _I, _P, _P, _P, _SZ, _P]),
    "gpsig_tens_vjp_workspace_bytes": (_SZ, [_I, _I, _I]),
    "gpsig_tens_vjp_wide_workspace_bytes": (_SZ, [_I, _I, _I, _I, _I]),
    "gpsig_tens_gram_vjp_workspace_bytes": (_SZ, [_I, _I, _I, _I, _I, _I]),
    "gpsig_tens_gram_vjp": (_I, [_P, _I, _I, _I, _I, _I, _I, _P, _P, _P, _SZ, _P]),
    "gpsig_rescaled": (_I, [_P, _I, _I, _P, _I, _I, _I, _I, _I, _P, _P, _SZ, _P]),
    "gpsig_rescaled_workspace_bytes": (_SZ, [_I, _I]),
    "gpsig_tens_workspace_bytes": (_SZ, [_I, _I, _I, _I, _I]),
    "gpsig_signature_channels": (ctypes.c_longlong, [_I, _I]),
    "gpsig_signature": (_I, [_P, _I, _I, _I, _I, _P, _P]),
    "gpsig_signature_vjp": (_I, [_P, _I, _I, _I, _I, _P, _P, _P]),
    "gpsig_signature_workspace_bytes": (_SZ, [_I, _I, _I, _I]),
    "gpsig_signature_ex": (_I, [_P, _I, _I, _I, _I, _P, _P, _SZ, _P]),
    "gpsig_signature_vjp_ex": (_I, [_P, _I, _I, _I, _I, _P, _P, _P, _SZ, _P]),
    "gpsig_gemm_f32": (_I, [_I, _I, _I, _I, _I, _F, _P, ctypes.c_longlong, _P, ctypes.c_longlong, _F, _P,
                            ctypes.c_longlong, _P]),
    "gpsig_gemm_splitk_bytes": (_SZ, [_I, _I, _I]),
    "gpsig_gemm_f32_splitk": (_I, [_I, _I, _I, _I, _I, _F, _P, ctypes.c_longlong, _P, ctypes.c_longlong, _F, _P,
                                   ctypes.c_longlong, _P, _SZ, _P]),
    "gpsig_version": (ctypes.c_char_p, []),
}

_lock = threading.Lock()
_lib = None


class GpsigError(RuntimeError):
    pass


def load():
    """Return the loaded library (raises GpsigError if it is missing or incomplete)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise GpsigError(f"gpsig_amd native library not found at {LIB_PATH}; build it with "
                             "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)")
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            try:
                fn = getattr(lib, name)
            except AttributeError as e:
                raise GpsigError(f"{LIB_PATH} does not export {name}") from e
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


def check(rc: int, what: str) -> None:
    if rc != GPSIG_OK:
        raise GpsigError(f"{what}: {_ERRORS.get(rc, 'error')} (code {rc})")
