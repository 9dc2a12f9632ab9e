"""ctypes binding of libraman_mi355x.so (the C ABI declared in include/raman_mi355x.h).

torch is imported first on purpose: the library is linked against the HIP runtime that
PyTorch-ROCm bundles (torch/lib/libamdhip64.so) and must resolve to that already-loaded copy so
that device pointers and streams are shared with torch.  There is no fallback: if the library is
missing the import fails loudly.
"""
import ctypes
import glob
import hashlib
import os

import torch  # noqa: F401  (must be loaded before the library, see module docstring)

PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG, "lib", "libraman_mi355x.so")
CSRC = os.path.join(os.path.dirname(PKG), "csrc")
HEADER = os.path.join(os.path.dirname(os.path.dirname(PKG)), "include", "raman_mi355x.h")

RDN_OK = 0
ABI_VERSION = 6
# exact metric accumulator words (include/raman_mi355x.h RDN_ACC_*)
ACC_LIMBS = 6
ACC_STRIDE = ACC_LIMBS + 1
ACC_COUNT = 4 * ACC_STRIDE
ACC_WORDS = ACC_COUNT + 1
ACC_FRAC_BITS = 128


def source_hash():
    """sha256 prefix of the sources the library is built from -- the same files, in the same order,
    as csrc/Makefile's STAMP_SRC (None when the sources are not beside the package)."""
    if not os.path.isdir(CSRC):
        return None
    files = sorted(os.path.basename(p) for pat in ("*.hip", "*.cpp", "*.hpp")
                   for p in glob.glob(os.path.join(CSRC, pat)))
    paths = [os.path.join(CSRC, f) for f in files] + [os.path.join(CSRC, "Makefile"), HEADER]
    h = hashlib.sha256()
    for p in paths:
        with open(p, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]

c_float_p = ctypes.POINTER(ctypes.c_float)
c_double_p = ctypes.POINTER(ctypes.c_double)


class GenParams(ctypes.Structure):
    _fields_ = [("signal_length", ctypes.c_int64), ("snr_lo", ctypes.c_float), ("snr_hi", ctypes.c_float),
                ("extreme_noise_prob", ctypes.c_float), ("max_repeat", ctypes.c_int32)]


_SIGNATURES = {
    "rdn_version": ([], ctypes.c_int),
    "rdn_build_id": ([], ctypes.c_char_p),
    "rdn_default_correction_mask": ([ctypes.c_int, ctypes.POINTER(ctypes.c_uint64)], ctypes.c_int),
    "rdn_get_correction_mask": ([ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
                                 ctypes.POINTER(ctypes.c_uint64)], ctypes.c_int),
    "rdn_forward_status": ([ctypes.c_int, ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p,
                            ctypes.c_size_t, ctypes.c_void_p], ctypes.c_int),
    "rdn_last_error": ([], ctypes.c_char_p),
    "rdn_param_names": ([ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)], ctypes.c_int),
    "rdn_packed_size": ([ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_size_t)], ctypes.c_int),
    "rdn_pack": ([ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_int64),
                  ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t], ctypes.c_int),
    "rdn_workspace_size": ([ctypes.c_int, ctypes.c_int, ctypes.c_int64, ctypes.c_int64,
                            ctypes.POINTER(ctypes.c_size_t), ctypes.c_void_p], ctypes.c_int),
    "rdn_workspace_init": ([ctypes.c_int, ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p,
                            ctypes.c_size_t, ctypes.c_void_p], ctypes.c_int),
    "rdn_check_blob": ([ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t], ctypes.c_int),
    "rdn_forward": ([ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                     ctypes.c_int64, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p], ctypes.c_int),
    "rdn_forward_metrics": ([ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                             ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                             ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                             ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
    "rdn_forward_status_ex": ([ctypes.c_int, ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p,
                               ctypes.c_size_t, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint)], ctypes.c_int),
    "rdn_generate": ([ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int64, ctypes.POINTER(GenParams), ctypes.c_void_p,
                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p], ctypes.c_int),
    "rdn_metrics": ([ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p,
                     ctypes.c_void_p, ctypes.c_void_p], ctypes.c_int),
    "rdn_metrics_ex": ([ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p,
                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p], ctypes.c_int),
    "rdn_acc_value": ([ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_double)], ctypes.c_int),
}

EXPORTED = tuple(_SIGNATURES)

_lib = None


def lib():
    """Load (once) and return the native library.  Raises ImportError if it is not built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"raman_mi355x native library not built: {LIB_PATH} is missing "
                              "(run `python -c 'import __graft_entry__ as g; g.build()'` or `make -C csrc`)")
        handle = ctypes.CDLL(LIB_PATH)
        for name, (args, res) in _SIGNATURES.items():
            fn = getattr(handle, name)
            fn.argtypes = args
            fn.restype = res
        if handle.rdn_version() != ABI_VERSION:
            raise ImportError(f"libraman_mi355x ABI {handle.rdn_version()} != expected {ABI_VERSION}")
        built, tree = handle.rdn_build_id().decode(), source_hash()
        if tree is not None and built != tree and os.environ.get("RDN_ALLOW_STALE_LIB") != "1":
            raise ImportError(f"stale libraman_mi355x.so: built from sources {built}, this tree's sources hash to "
                              f"{tree}; rebuild it (make -C csrc, or __graft_entry__.build())")
        _lib = handle
    return _lib


RDN_ERANGE = -6


class EngineError(RuntimeError):
    pass


class RangeError(EngineError):
    """RDN_ERANGE: an RDN_F16F8 / RDN_F16MIX activation left the e4m3 correction planes' range (the
    affected tiles' outputs are NaN); RDN_F32 / RDN_BF16X3 have no such bound."""


def check(rc, what):
    if rc != RDN_OK:
        msg = lib().rdn_last_error().decode(errors="replace")
        raise (RangeError if rc == RDN_ERANGE else EngineError)(f"{what} failed (code {rc}): {msg}")
