"""The C-ABI library loads and exports everything include/gpfit.h declares (no GPU needed)."""
import ctypes
import re

import pytest

from conftest import ROOT


def _declared():
    hdr = (ROOT / "include" / "gpfit.h").read_text()
    return sorted(set(re.findall(r"\b(gpf_[a-z_0-9]+)\s*\(", hdr)))


def test_library_exports_every_declared_symbol():
    import gpfit._lib as L
    lib = L.load_library()
    names = _declared()
    assert len(names) >= 14
    for n in names:
        assert getattr(lib, n) is not None, n
    # the ctypes signature table covers the header exactly
    assert sorted(L.SIGNATURES) == names


def test_abi_version_and_tile():
    import gpfit._lib as L
    lib = L.load_library()
    assert lib.gpf_version() == L.ABI_VERSION == 2
    assert lib.gpf_tile() == 128


def test_library_was_built_from_these_sources():
    """gpf_build_info carries the source hash __graft_entry__.build() compiled it from: the
    library every test loads is the one built from this tree."""
    import __graft_entry__ as ge
    import gpfit
    info = gpfit.build_info()
    assert info.startswith(f"src={ge.source_hash()};hipcc="), (info, ge.source_hash())


def test_library_is_gfx950_code_object():
    import subprocess
    so = ROOT / "gaussian-process_amd" / "libgpfit.so"
    out = subprocess.run(["/opt/rocm/bin/roc-obj-ls", str(so)], capture_output=True, text=True)
    if out.returncode != 0:
        pytest.skip("roc-obj-ls unavailable")
    assert "gfx950" in out.stdout


def test_no_cpu_fallback_without_device():
    """The product path must fail loudly when no GPU is visible."""
    import gpfit._lib as L
    lib = L.load_library()
    n = ctypes.c_int(0)
    h = ctypes.c_void_p()
    if lib.gpf_open(0, ctypes.byref(h)) == 0:
        lib.gpf_close(h)
        pytest.skip("a GPU is visible")
    with pytest.raises(L.GPFitError):
        L.Context(0)
    import GP_func
    import numpy as np
    with pytest.raises(L.GPFitError):
        GP_func.GP(np.zeros((1, 3)), np.zeros(3), np.ones(3), np.zeros((1, 3)), np.ones(1))
    del n


def test_bad_arguments_are_value_errors_without_touching_device():
    import gpfit._lib as L
    lib = L.load_library()
    assert lib.gpf_set_data(None, None, None, None, 0, 0) == L.GPF_BAD_ARG
    assert lib.gpf_eval_batch(None, None, 0, None, None, None, None) == L.GPF_BAD_ARG


def test_comm_transport_codes():
    """INTEGRATION.md's fallback: the host transport is GPF_COMM_HOST = 2 (RCCL = 1); any other
    code, 0 included, is rejected with GPF_BAD_ARG before any socket or device is touched."""
    import gpfit._lib as L
    lib = L.load_library()
    assert (L.GPF_COMM_RCCL, L.GPF_COMM_HOST) == (1, 2)
    out = ctypes.c_void_p()
    for bad in (0, 3, -1):
        assert lib.gpf_comm_open(None, 0, 1, b"127.0.0.1", 29999, bad, ctypes.byref(out)) == L.GPF_BAD_ARG
        assert not out.value
    # one rank over the host transport needs no rendezvous: opens, exchanges, closes
    assert lib.gpf_comm_open(None, 0, 1, b"127.0.0.1", 29999, L.GPF_COMM_HOST, ctypes.byref(out)) == L.GPF_OK
    assert out.value
    lib.gpf_comm_close(out)
