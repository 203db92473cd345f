"""CPU: the 64-bit-limb CPU baseline (tests/hostemu/cpu64_verify.cpp, bench.py's
cpu_baseline main leg) gives the golden verdict codes and Gt bytes
(tests/golden/vectors.json, oracle-generated and pinned by the reference KATs)
and the golden hash_to_g1 points; its constants header is what the generator
produces from the oracle today."""
import ctypes
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HE = os.path.join(ROOT, "tests", "hostemu")
P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB


@pytest.fixture(scope="module")
def lib():
    src, hdr = os.path.join(HE, "cpu64_verify.cpp"), os.path.join(HE, "cpu64_consts.h")
    so = os.path.join(HE, "libcpu64_verify.so")
    if not os.path.exists(so) or os.path.getmtime(so) < max(os.path.getmtime(src), os.path.getmtime(hdr)):
        subprocess.check_call(["g++", "-O3", "-std=c++17", "-shared", "-fPIC", "-pthread", src, "-o", so])
    return ctypes.CDLL(so)


def test_consts_header_is_generated():
    out = subprocess.check_output([sys.executable, os.path.join(HE, "gen_cpu64_consts.py")], text=True)
    with open(os.path.join(HE, "cpu64_consts.h")) as f:
        assert f.read().strip() == out.strip()


def test_golden_codes_and_gt(lib, vectors):
    n = 0
    for c in vectors["cases"]:
        sig, msg, pk = bytes.fromhex(c["sig"]), bytes.fromhex(c["msg"]), bytes.fromhex(c["pk"])
        if len(sig) != 48 or len(pk) != 96:
            continue   # length codes are decided before any arithmetic
        gt = (ctypes.c_uint8 * 576)()
        code = lib.cpu64_gt(sig, msg, ctypes.c_uint64(len(msg)), pk, gt)
        assert code == c["code"], c["name"]
        if "gt" in c:
            assert bytes(gt).hex() == c["gt"], c["name"]
        n += 1
    assert n >= 40


def test_hash_to_g1(lib, vectors):
    for h in vectors["hash_to_g1"]:
        msg = bytes.fromhex(h["msg"])
        out = (ctypes.c_uint8 * 96)()
        assert lib.cpu64_hash(msg, ctypes.c_uint64(len(msg)), out) == 0
        x = int.from_bytes(bytes(out[:48]), "big")
        y = int.from_bytes(bytes(out[48:]), "big")
        comp = bytearray(x.to_bytes(48, "big"))
        comp[0] |= 0x80 | (0x20 if y > (P - 1) // 2 else 0)
        assert bytes(comp).hex() == h["h"]


def test_batch_threads(lib, vectors):
    cases = [c for c in vectors["cases"] if len(c["sig"]) == 96 and len(c["pk"]) == 192]
    cases = (cases * 3)[:100]
    sigs = b"".join(bytes.fromhex(c["sig"]) for c in cases)
    pks = b"".join(bytes.fromhex(c["pk"]) for c in cases)
    msgs = [bytes.fromhex(c["msg"]) for c in cases]
    offs = [0]
    for m in msgs:
        offs.append(offs[-1] + len(m))
    o = (ctypes.c_uint64 * len(offs))(*offs)
    codes = (ctypes.c_uint8 * len(cases))()
    lib.cpu64_verify_batch(ctypes.c_uint64(len(cases)), sigs, pks, b"".join(msgs), o, codes, 4)
    assert list(codes) == [c["code"] for c in cases]
