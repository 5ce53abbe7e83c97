"""CPU: the drop-in boundary.  libringo.so loads without a GPU and exports exactly the symbols
include/ringo.h declares; host-side argument checks return the reference's error codes
without touching the device; the Python mirror raises the reference's panic messages."""
import ctypes

import numpy as np
import pytest

import ringo
from ringo import _lib


def test_library_exports_every_header_symbol():
    lib = _lib.lib()
    names = _lib.header_symbols()
    assert len(names) >= 30
    for n in names:
        assert hasattr(lib, n), n
    # and nothing in the binding table is missing from the header
    assert set(_lib._SIGS) <= set(names)


def test_version_names_sampler_layout():
    """rg_version ends in the build's sampler layout (include/ringo.h RG_SAMPLER_LAYOUT): round 5
    renumbered the COSAC instances (groups of 8), so sampled commitments differ from layout 1's."""
    import re
    m = re.search(r"#define RG_SAMPLER_LAYOUT (\d+)", open(_lib.HEADER).read())
    assert m and int(m.group(1)) == 2
    v = _lib.lib().rg_version().decode()
    assert v.startswith("libringo 0.2 gfx950") and v.endswith("sampler-layout " + m.group(1)), v


def test_status_strings_match_reference_panics():
    L = _lib.lib()
    assert L.rg_status_string(-1) == b"inconsistent input(s)"
    assert L.rg_status_string(-2) == b"rank must be a power of two"
    assert L.rg_status_string(-3) == b"NTT not supported"
    assert L.rg_status_string(-6) == b"len(v) > params.rank"


def test_field_create_and_constants_no_gpu(fields):
    F = ringo.Field(fields["jindo_zp"])
    qinv, r2, one = F.constants()
    assert qinv == 18446744073709551615  # element.go:72
    assert int(r2[0]) == 17372242133975344483  # element.go:785


def test_transformer_argument_errors_no_gpu(fields):
    F = ringo.Field(fields["p63"])
    with pytest.raises(ringo.RingoPanic, match="power of two"):
        ringo.CyclotomicTransformer(F, 12)
    G = ringo.Field(97)  # 97 - 1 = 2^5 * 3: 2N | q-1 fails for N = 32
    with pytest.raises(ringo.RingoPanic, match="NTT not supported"):
        ringo.CyclotomicTransformer(G, 32)
    with pytest.raises(ringo.RingoPanic, match="NTT not supported"):
        ringo.CyclicTransformer(G, 64)


def test_evaluator_domain_panics_no_gpu(fields):
    F = ringo.Field(fields["p63"])

    class _NoNTT:  # never reached: checks run before any device call
        pass

    ev = ringo.bigpoly.CyclotomicEvaluator(F, 8, _NoNTT())
    a, b = ev.NewPoly(False), ev.NewPoly(True)
    with pytest.raises(ringo.RingoPanic, match="inconsistent input"):
        ev.AddTo(ev.NewPoly(False), a, b)
    with pytest.raises(ringo.RingoPanic, match="not in NTT domain"):
        ev.MulTo(ev.NewPoly(True), a, a)
    with pytest.raises(ringo.RingoPanic, match="already in NTT domain"):
        ev.NTTTo(ev.NewPoly(True), b)
    with pytest.raises(ringo.RingoPanic, match="input not in NTT domain"):
        ev.InvNTTTo(ev.NewPoly(False), a)
    with pytest.raises(ringo.RingoPanic, match="inconsistent input"):
        ev.NegTo(ringo.Poly(F, 16), a)


def test_null_handles_rejected_no_gpu():
    L = _lib.lib()
    assert L.rg_ntt_fwd(None, None, None, 1) == -1
    assert L.rg_vec(None, 0, None, None, None, 1) == -1
    assert L.rg_jindo_commit(None, None, 0, None, None, None, None, None, None, None, None) == -1
    h = ctypes.c_void_p()
    assert L.rg_field_create(1, _lib.ptr(np.array([4], np.uint64)), ctypes.byref(h)) == -1  # even modulus


def test_production_library_refuses_probe_no_gpu():
    """libringo.so has no measurement switch: rg_set_probe refuses every probe but 0, and no
    source of the product reads the environment (the RINGO_* kernel switches live only in the
    experiments build, tools/experiments/knobs_env.hip)."""
    L = _lib.lib()
    for probe in (1, 4, 5, -1):
        assert L.rg_set_probe(probe) == -1  # RG_ERR_INVALID
    assert L.rg_set_probe(0) == 0
    import glob
    import os
    csrc = os.path.join(os.path.dirname(_lib._ROOT), "ringo-snark_amd", "csrc")
    for fn in glob.glob(os.path.join(csrc, "*")):
        assert "getenv" not in open(fn).read(), fn


def test_experiments_library_honours_probe_no_gpu():
    """libringo_exp.so: the same ABI, probes 4 and 5 accepted (per calling thread), others not."""
    import threading
    E = _lib.load(_lib.EXP_LIB_PATH)
    assert E.rg_set_probe(4) == 0
    assert E.rg_set_probe(5) == 0
    assert E.rg_set_probe(3) == -1
    seen = []
    t = threading.Thread(target=lambda: seen.append(E.rg_set_probe(0)))
    t.start()
    t.join()
    assert seen == [0]
    assert E.rg_set_probe(0) == 0
    for n in _lib.header_symbols():
        assert hasattr(E, n), n


def test_mac_kinds_argument_errors_no_gpu():
    L = _lib.lib()
    a, b = ctypes.c_int(), ctypes.c_int()
    assert L.rg_jindo_mac_kinds(None, ctypes.byref(a), ctypes.byref(b)) == -1
