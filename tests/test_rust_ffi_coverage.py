"""CPU: the Rust host crate's FFI layer (utils/verify-bls-signatures-gpu/src/
ffi.rs) declares every function of the C ABI headers (include/cess_bls.h,
include/cess_rsa.h), with the same parameter count, so DESIGN.md's "ffi.rs
binds every header entry point" stays true as the ABI grows.  (No cargo in
this image: a text check, not a compile.)"""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_functions():
    funcs = {}
    for h in ("cess_bls.h", "cess_rsa.h"):
        text = open(os.path.join(ROOT, "include", h)).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        for m in re.finditer(r"\b(cess_(?:bls|rsa)_[a-z0-9_]+)\s*\(([^;{]*?)\)\s*;", text):
            args = m.group(2).strip()
            funcs[m.group(1)] = 0 if args in ("", "void") else args.count(",") + 1
    return funcs


def _rust_functions():
    text = open(os.path.join(ROOT, "utils", "verify-bls-signatures-gpu", "src", "ffi.rs")).read()
    funcs = {}
    for m in re.finditer(r"pub fn (cess_(?:bls|rsa)_[a-z0-9_]+)\s*\((.*?)\)\s*(?:->[^;]*)?;", text, flags=re.S):
        args = m.group(2).strip().rstrip(",")
        funcs[m.group(1)] = 0 if not args else args.count(",") + 1
    return funcs


def test_every_header_function_is_bound_in_rust():
    h, r = _header_functions(), _rust_functions()
    assert len(h) > 50
    missing = sorted(set(h) - set(r))
    assert not missing, missing
    wrong = sorted(f for f in h if h[f] != r[f])
    assert not wrong, [(f, h[f], r[f]) for f in wrong]
