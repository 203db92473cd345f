"""CPU: the C-ABI library (cess_amd/lib/libcess_bls.so) loads and exports every
symbol include/cess_bls.h declares; without a GPU it fails loudly (no CPU fallback)."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "cess_amd", "lib", "libcess_bls.so")


def header_symbols():
    txt = ""
    for h in ("cess_bls.h", "cess_rsa.h"):
        with open(os.path.join(ROOT, "include", h)) as f:
            txt += f.read()
    return sorted(set(re.findall(r"\b(cess_(?:bls|rsa)_[a-z0-9_]+)\s*\(", txt)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        subprocess.check_call(["make", "-C", os.path.join(ROOT, "cess_amd", "csrc"), "-j8"])
    return ctypes.CDLL(LIB)


def test_exports_every_header_symbol(lib):
    syms = header_symbols()
    assert len(syms) >= 13
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    from cess_amd import bls
    assert sorted(bls.EXPORTS) == syms


def test_status_strings(lib):
    lib.cess_bls_status_string.restype = ctypes.c_char_p
    assert b"CPU fallback" in lib.cess_bls_status_string(-2)
    lib.cess_bls_version.restype = ctypes.c_char_p
    assert b"gfx950" in lib.cess_bls_version()


def test_no_device_fails_loudly(lib):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from cess_amd import bls
    with pytest.raises(bls.DeviceUnavailable):
        bls.Context()
