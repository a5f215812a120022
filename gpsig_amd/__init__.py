"""gpsig_amd -- MI355X-native signature-kernel Gram evaluator (drop-in for the hot path of GPSig).

Python host on PyTorch-ROCm tensors; the recursions run in hand-written gfx950 HIP kernels from
``libgpsig_amd.so`` behind the C ABI in ``include/gpsig_amd.h``.
"""
from . import kernels, kernels_pde, ops  # noqa: F401
from ._lib import GpsigError, load  # noqa: F401
from .kernels import (SignatureKernel, SignatureLinear, SignatureRBF, SignatureGauss)  # noqa: F401
from .kernels_pde import UntruncSignatureKernel  # noqa: F401

__version__ = "0.1.0"
