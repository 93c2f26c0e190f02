"""ctypes binding of ``libdkg.so`` (C ABI in ``include/dkg.h``).

The library is the product: there is no CPU fallback.  Loading fails loudly
when the shared object is missing, and every entry point raises on a non-zero
status with the library's own message.
"""

from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_double, c_float, c_int, c_int32, c_size_t, c_void_p

from .errors import BotorchTensorDimensionError, DkgNativeError, NotPSDError, UnsupportedError

# DKG_LIB: an alternative build of the same library (A/B measurements by tools/; never set in production)
LIB_PATH = os.environ.get("DKG_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "_native",
                                                     "libdkg.so")

ABI_VERSION = 8
DKG_XARG_MAX = 64  # include/dkg.h: largest B * d of dkg_plan_forward_grad_hostx
DKG_PLAN_GRAD = 1
DKG_PLAN_FORCE_WALK = 2  # test hook: envelope overflow path for every pair
DKG_PLAN_F32 = 4  # fp32 contractions (BASELINE configs[4]); forward only
DKG_PLAN_FUSED = 8  # the forward as one launch with in-launch hand-offs (dkg_fused.h); not the default
DKG_PLAN_NO_CHAIN = 16  # test hook: the streaming envelope's list-overflow path (no sample chain) for every pair
# dkg_debug_cov_kernels: the opt-in fp64 covariance block kernels (same bits as the defaults)
DKG_COV_ENABLE_BLK, DKG_COV_ENABLE_REC2, DKG_COV_ENABLE_REG = 1, 2, 4
MAX_OUTPUTS = 8
MAX_DIM = 16

(DKG_OK, DKG_ERR_ARG, DKG_ERR_UNSUPPORTED, DKG_ERR_WORKSPACE, DKG_ERR_HIP, DKG_ERR_NO_LINES,
 DKG_ERR_NOT_PD) = range(7)


class DkgOutput(ctypes.Structure):
    """``struct dkg_output`` (include/dkg.h)."""

    _fields_ = [
        ("n", c_int32),
        ("kernel", c_int32),
        ("outputscale", c_double),
        ("noise", c_double),
        ("mean_constant", c_double),
        ("y_mean", c_double),
        ("y_std", c_double),
        ("inv_lengthscale", c_void_p),
        ("train_x", c_void_p),
        ("alpha", c_void_p),
        ("root_frag", c_void_p),
        ("disc_frag", c_void_p),
        ("disc_mean", c_void_p),
    ]


# name -> (restype, argtypes); every symbol include/dkg.h declares.
SIGNATURES = {
    "dkg_abi_version": (c_int, []),
    "dkg_last_error": (c_char_p, []),
    "dkg_frag_elems": (c_size_t, [c_int, c_int]),
    "dkg_kernel_matrix": (c_int, [POINTER(DkgOutput), c_int, c_void_p, c_int, c_void_p, c_int, c_double,
                                  c_void_p, c_void_p]),
    "dkg_pack_root": (c_int, [c_void_p, c_int, c_void_p, c_void_p]),
    "dkg_prepare_workspace": (c_size_t, [c_int]),
    "dkg_prepare_output": (c_int, [POINTER(DkgOutput), c_int, c_void_p, c_int, c_void_p, c_void_p, c_size_t,
                                   c_void_p, c_void_p, POINTER(c_double), c_void_p]),
    "dkg_prepare_outputs": (c_int, [POINTER(DkgOutput), c_int, c_int, POINTER(c_void_p), c_int, POINTER(c_void_p),
                                    POINTER(c_void_p), POINTER(c_size_t), POINTER(c_void_p), POINTER(c_void_p),
                                    POINTER(c_double), c_void_p]),
    "dkg_cross_root": (c_int, [POINTER(DkgOutput), c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p]),
    "dkg_forward_workspace": (c_size_t, [POINTER(DkgOutput), c_int, c_int, c_int, c_int]),
    "dkg_forward": (c_int, [POINTER(DkgOutput), c_int, c_int, c_void_p, c_int, c_void_p, c_int, c_void_p, c_int,
                            c_int, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "dkg_forward_timed": (c_int, [POINTER(DkgOutput), c_int, c_int, c_void_p, c_int, c_void_p, c_int, c_void_p,
                                  c_int, c_int, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p,
                                  POINTER(c_float)]),
    "dkg_plan_bytes": (c_size_t, []),
    "dkg_plan_workspace": (c_size_t, [POINTER(DkgOutput), c_int, c_int, c_int, c_int, c_int, c_int]),
    "dkg_plan_init": (c_int, [POINTER(DkgOutput), c_int, c_int, c_void_p, c_int, c_void_p, c_int, c_int, c_int,
                              c_int, c_void_p, c_size_t, c_void_p, c_void_p, c_void_p]),
    "dkg_plan_forward_grad": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p]),
    "dkg_plan_forward_grad_hostx": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p,
                                            c_void_p, c_void_p]),
    "dkg_plan_forward": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p]),
    "dkg_plan_forward_batches": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p]),
    "dkg_plan_forward_timed": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p,
                                       POINTER(c_float)]),
    "dkg_plan_time_stage": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int,
                                    c_int, POINTER(c_float)]),
    "dkg_plan_time_stage_batches": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_int,
                                            c_int, POINTER(c_float)]),
    "dkg_plan_hull_sizes": (c_int, [c_void_p, c_void_p, c_int, c_void_p]),
    "dkg_plan_status": (c_int, [c_void_p, POINTER(c_int), c_int, c_void_p]),
    "dkg_plan_fused": (c_int, [c_void_p]),
    "dkg_lines_kg": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "dkg_epigraph": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
    "dkg_pwl_expectation": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p]),
    "dkg_plan_lines": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p]),
    "dkg_launcher_create": (c_int, [c_int, POINTER(c_void_p)]),
    "dkg_launcher_arm": (c_int, [c_void_p, c_double]),
    "dkg_launcher_graphs": (c_int, [c_void_p, c_int, POINTER(c_void_p), POINTER(c_int), POINTER(c_void_p)]),
    "dkg_launcher_destroy": (c_int, [c_void_p]),
    "dkg_debug_read_kstamps": (c_int, [c_void_p, c_int]),
    "dkg_debug_wave_ops": (c_int, [c_void_p, c_void_p, c_void_p]),
    "dkg_debug_cov_kernels": (c_int, [c_int]),
    "dkg_debug_mfma_f64": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p]),
}

_lib = None


def load() -> ctypes.CDLL:
    """Load and type the native library once (raises DkgNativeError if absent)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise DkgNativeError(
            f"libdkg.so not found at {LIB_PATH}; build it with `make -C decoupled-kg_amd` "
            f"(or __graft_entry__.build()).  There is no CPU fallback.")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.dkg_abi_version() != ABI_VERSION:
        raise DkgNativeError(f"libdkg.so ABI {lib.dkg_abi_version()} != expected {ABI_VERSION}; rebuild it")
    _lib = lib
    return lib


def check(status: int, what: str) -> None:
    if status == DKG_OK:
        return
    msg = f"{what}: {load().dkg_last_error().decode(errors='replace')}"
    if status == DKG_ERR_ARG:
        raise BotorchTensorDimensionError(msg)
    if status == DKG_ERR_UNSUPPORTED:
        raise UnsupportedError(msg)
    if status == DKG_ERR_NO_LINES:
        raise ValueError(msg)
    if status == DKG_ERR_NOT_PD:
        raise NotPSDError(msg)
    raise DkgNativeError(msg)


def ptr(t) -> int:
    """Device address of a tensor (0 for None)."""
    return 0 if t is None else int(t.data_ptr())
