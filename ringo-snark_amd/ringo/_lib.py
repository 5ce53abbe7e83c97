"""ctypes loader for libringo.so (the HIP library).  The product path has no fallback: if the
library is missing or fails to load, every call raises ("no CPU fallback")."""
import ctypes
import os
import re

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# RINGO_LIB: another build of the same ABI (tools/: profiling variants, the experiments build)
LIB_PATH = os.environ.get("RINGO_LIB") or os.path.join(_ROOT, "lib", "libringo.so")
# the experiments build (ringo-snark_amd/Makefile): RINGO_* kernel switches and rg_set_probe honoured;
# RINGO_EXP_LIB: an experiments-build variant (tools/var_build.sh exp_<name>)
EXP_LIB_PATH = os.environ.get("RINGO_EXP_LIB") or os.path.join(_ROOT, "lib", "libringo_exp.so")
HEADER = os.path.join(os.path.dirname(_ROOT), "include", "ringo.h")

u64p = ctypes.POINTER(ctypes.c_uint64)
i64p = ctypes.POINTER(ctypes.c_int64)
vp = ctypes.c_void_p

_lib = None


class RingoError(RuntimeError):
    """A libringo call failed.  `message` holds the reference's panic text where one exists
    (e.g. "inconsistent input(s)", "NTT not supported")."""

    def __init__(self, status, message, detail=""):
        super().__init__(message + (f" ({detail})" if detail else ""))
        self.status = status
        self.message = message


class JindoStddevsC(ctypes.Structure):
    _fields_ = [(n, ctypes.c_double) for n in ["ecd", "ecd_blind", "mask", "mask_blind", "mlwe", "mask_mlwe"]]


class JindoSeedsC(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint8 * 32) for n in ["enc_cdt", "enc_cosac", "enc_cosac_round", "mlwe_cdt",
                                                     "mlwe_round", "uniform"]]


class JindoParamsC(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in
                ["rank", "rows", "cols", "slots", "exp", "d", "in_msis", "out_msis", "mlwe", "dcmp",
                 "log_in_cut", "log_out_cut"]] + [
        ("base", ctypes.c_uint64), ("nq", ctypes.c_int), ("nqo", ctypes.c_int),
        ("q", ctypes.c_uint64 * 4), ("qo", ctypes.c_uint64 * 4), ("field_limbs", ctypes.c_int),
        ("field_q", ctypes.c_uint64 * 16)]


_SIGS = {
    "rg_status_string": (ctypes.c_char_p, [ctypes.c_int]),
    "rg_last_error": (ctypes.c_char_p, []),
    "rg_version": (ctypes.c_char_p, []),
    "rg_field_create": (ctypes.c_int, [ctypes.c_int, u64p, ctypes.POINTER(vp)]),
    "rg_field_destroy": (None, [vp]),
    "rg_field_limbs": (ctypes.c_int, [vp]),
    "rg_field_constants": (ctypes.c_int, [vp, u64p, u64p, u64p]),
    "rg_ntt_create": (ctypes.c_int, [vp, ctypes.c_int, ctypes.c_int, ctypes.POINTER(vp)]),
    "rg_ntt_create_from_tables": (ctypes.c_int, [vp, ctypes.c_int, ctypes.c_int, u64p, u64p, u64p,
                                                 ctypes.POINTER(vp)]),
    "rg_ntt_destroy": (None, [vp]),
    "rg_ntt_rank": (ctypes.c_int, [vp]),
    "rg_ntt_tables": (ctypes.c_int, [vp, u64p, u64p, u64p]),
    "rg_ntt_fwd": (ctypes.c_int, [vp, u64p, u64p, ctypes.c_size_t]),
    "rg_ntt_fwd_dev": (ctypes.c_int, [vp, vp, vp, ctypes.c_size_t, vp]),
    "rg_ntt_inv": (ctypes.c_int, [vp, u64p, u64p, ctypes.c_size_t]),
    "rg_ntt_inv_dev": (ctypes.c_int, [vp, vp, vp, ctypes.c_size_t, vp]),
    "rg_vec": (ctypes.c_int, [vp, ctypes.c_int, u64p, u64p, u64p, ctypes.c_size_t]),
    "rg_vec_dev": (ctypes.c_int, [vp, ctypes.c_int, vp, vp, vp, ctypes.c_size_t, vp]),
    "rg_poly_quorem_vanishing_dev": (ctypes.c_int, [vp, ctypes.c_size_t, ctypes.c_longlong, vp, vp, vp,
                                                    ctypes.c_size_t, vp]),
    "rg_poly_quorem_vanishing": (ctypes.c_int, [vp, ctypes.c_size_t, ctypes.c_longlong, u64p, u64p, u64p]),
    "rg_poly_aut_dev": (ctypes.c_int, [vp, ctypes.c_size_t, ctypes.c_longlong, ctypes.c_int, vp, vp, ctypes.c_size_t,
                                       vp]),
    "rg_poly_aut": (ctypes.c_int, [vp, ctypes.c_size_t, ctypes.c_longlong, ctypes.c_int, u64p, u64p]),
    "rg_poly_evaluate_dev": (ctypes.c_int, [vp, vp, ctypes.c_size_t, vp, vp, vp, vp]),
    "rg_poly_evaluate_scratch_bytes": (ctypes.c_size_t, [vp, ctypes.c_size_t]),
    "rg_poly_evaluate": (ctypes.c_int, [vp, u64p, ctypes.c_size_t, u64p, u64p]),
    "rg_poly_modswitch_dev": (ctypes.c_int, [vp, ctypes.c_size_t, vp, ctypes.c_size_t, u64p, vp, vp]),
    "rg_poly_modswitch": (ctypes.c_int, [vp, ctypes.c_size_t, u64p, ctypes.c_size_t, u64p, u64p]),
    "rg_buckler_encode_dev": (ctypes.c_int, [vp, ctypes.c_size_t, vp, vp, ctypes.c_size_t, vp, vp, vp]),
    "rg_buckler_encode_scratch_bytes": (ctypes.c_size_t, [vp, ctypes.c_size_t]),
    "rg_buckler_encode": (ctypes.c_int, [vp, ctypes.c_size_t, u64p, u64p, u64p]),
    "rg_buckler_circuit_create": (ctypes.c_int, [vp, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t), u64p,
                                                 ctypes.POINTER(ctypes.c_longlong), ctypes.POINTER(ctypes.c_size_t),
                                                 u64p, ctypes.POINTER(vp)]),
    "rg_buckler_circuit_destroy": (None, [vp]),
    "rg_buckler_eval_circuit_dev": (ctypes.c_int, [vp, ctypes.c_size_t, vp, vp, ctypes.c_size_t, vp, ctypes.c_size_t,
                                                   vp, vp]),
    "rg_buckler_eval_circuit": (ctypes.c_int, [vp, ctypes.c_size_t, u64p, u64p, ctypes.c_size_t, u64p,
                                               ctypes.c_size_t, u64p]),
    "rg_jindo_create": (ctypes.c_int, [ctypes.POINTER(JindoParamsC), u64p, u64p, u64p, ctypes.POINTER(vp)]),
    "rg_jindo_create_from_crs": (ctypes.c_int, [ctypes.POINTER(JindoParamsC), ctypes.c_char_p, ctypes.c_size_t,
                                                ctypes.POINTER(vp)]),
    "rg_jindo_create_dev": (ctypes.c_int, [ctypes.POINTER(JindoParamsC), vp, vp, vp, vp, ctypes.POINTER(vp)]),
    "rg_jindo_commit_key_dev": (ctypes.c_int, [vp, ctypes.POINTER(vp), ctypes.POINTER(vp), ctypes.POINTER(vp)]),
    "rg_jindo_commit_core": (ctypes.c_int, [vp, u64p, u64p, u64p, u64p]),
    "rg_jindo_commit_core_dev": (ctypes.c_int, [vp, ctypes.c_size_t, vp, vp, vp, vp, vp]),
    "rg_jindo_destroy": (None, [vp]),
    "rg_jindo_set_stddevs": (ctypes.c_int, [vp, ctypes.POINTER(JindoStddevsC)]),
    "rg_jindo_delta_inv": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_double)]),
    "rg_jindo_sample_dev": (ctypes.c_int, [vp, ctypes.c_size_t, vp, ctypes.c_size_t, ctypes.POINTER(JindoSeedsC),
                                           ctypes.c_ulonglong, vp, vp, vp, vp, vp]),
    "rg_jindo_commit_sampled_dev": (ctypes.c_int, [vp, ctypes.c_size_t, vp, ctypes.c_size_t,
                                                   ctypes.POINTER(JindoSeedsC), ctypes.c_ulonglong, vp, vp, vp, vp,
                                                   vp]),
    "rg_uniform_words_dev": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_ulonglong, ctypes.c_ulonglong,
                                            ctypes.c_size_t, vp, vp]),
    "rg_jindo_commit_key": (ctypes.c_int, [vp, u64p, u64p, u64p]),
    "rg_jindo_commit": (ctypes.c_int, [vp, u64p, ctypes.c_size_t, u64p, u64p, i64p, i64p, u64p, u64p, u64p, u64p]),
    "rg_jindo_commit_dev": (ctypes.c_int, [vp, ctypes.c_size_t, vp, ctypes.c_size_t, vp, vp, vp, vp, vp, vp, vp, vp,
                                           vp]),
    "rg_jindo_scratch_bytes": (ctypes.c_size_t, [vp, ctypes.c_size_t]),
    "rg_jindo_release_stream": (ctypes.c_int, [vp, vp]),
    "rg_jindo_mac_kinds": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
    "rg_jindo_eval_batch_dev": (ctypes.c_int, [vp, ctypes.c_size_t, vp, vp, vp, vp, vp, vp, vp, vp, vp]),
    "rg_jindo_eval_partial_dev": (ctypes.c_int, [vp, vp, vp, vp, vp]),
    "rg_jindo_eval_reduce_dev": (ctypes.c_int, [vp, vp, vp, vp, vp]),
    "rg_jindo_eval_respond_dev": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, vp]),
    "rg_jindo_verify_dev": (ctypes.c_int, [vp, ctypes.c_size_t] + [vp] * 11 + [ctypes.c_double, ctypes.c_double, vp,
                                                                            vp]),
    "rg_malloc": (ctypes.c_int, [ctypes.POINTER(vp), ctypes.c_size_t]),
    "rg_free": (ctypes.c_int, [vp]),
    "rg_memcpy_h2d": (ctypes.c_int, [vp, vp, ctypes.c_size_t, vp]),
    "rg_memcpy_d2h": (ctypes.c_int, [vp, vp, ctypes.c_size_t, vp]),
    "rg_memcpy_d2d": (ctypes.c_int, [vp, vp, ctypes.c_size_t, vp]),
    "rg_stream_sync": (ctypes.c_int, [vp]),
    "rg_set_device": (ctypes.c_int, [ctypes.c_int]),
    "rg_get_device": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
    "rg_set_probe": (ctypes.c_int, [ctypes.c_int]),
    "rg_device_count": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
}


def header_symbols():
    """Every function name declared in include/ringo.h."""
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(rg_[a-z0-9_]+)\s*\(", src)) - {"rg_status"})


def load(path):
    """A libringo build at `path` with every ABI signature set (a second, independent copy when
    `path` differs from the loaded product library: bench.py loads the experiments build this way
    for its compute-floor legs)."""
    try:
        import torch  # noqa: F401  (see lib())
    except ImportError:
        pass
    if not os.path.exists(path):
        raise RuntimeError(f"{path} not built: run __graft_entry__.build()")
    L = ctypes.CDLL(path)
    for name, (res, args) in _SIGS.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    return L


def lib():
    global _lib
    if _lib is None:
        # One HIP runtime per process: torch-ROCm bundles its own libamdhip64 (SONAME
        # libamdhip64.so.7).  Loading torch first makes libringo's NEEDED entry resolve to
        # that same copy, so device pointers and streams are shared; loading libringo first
        # would start /opt/rocm's runtime and torch would then fail to see any GPU.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"libringo.so not built at {LIB_PATH}: run __graft_entry__.build() "
                               "(there is no CPU fallback for the product path)")
        _lib = load(LIB_PATH)
    return _lib


def check(status):
    if status != 0:
        L = lib()
        msg = L.rg_status_string(status).decode()
        detail = L.rg_last_error().decode() if status in (-1, -3, -4) else ""
        raise RingoError(status, msg, detail)
    return status


def ptr(a):
    """numpy uint64 array -> POINTER(c_uint64)"""
    return None if a is None else a.ctypes.data_as(u64p)


def iptr(a):
    return None if a is None else a.ctypes.data_as(i64p)
