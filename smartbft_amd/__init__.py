"""smartbft_amd — MI355X-native signature verification behind SmartBFT's api.Verifier.

Layout:
  csrc/        HIP kernels for gfx950 (P-256 ECDSA verify, SHA-256) + the C-ABI host runtime
               -> libsbft_gpuverify.so (include/sbft_gpuverify.h)
  gpuverify.py ctypes binding of that C ABI (no CPU fallback)
"""
from .gpuverify import GpuVerifier, GpuVerifyError, PinnedArray, load_library  # noqa: F401
