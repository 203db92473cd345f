"""RSA PKCS#1 v1.5 raw verify (cp_enclave_verify::verify_rsa,
/root/reference/primitives/enclave-verify/src/lib.rs:221-228).

CPU: the oracle (oracle/rsa_oracle.py) reproduces every committed fixture
(tests/golden/rsa_vectors.json) and the reference test's round trip
(`cryptos_rsa`, enclave-verify/src/lib.rs:242-255: sign "hello world!" with
Pkcs1v15Sign::new_raw(), verify -> true); the library's host-side DER parser
agrees with the oracle on every good and malformed key.  Parity is unpinned
(no fixed vector in the reference; the rsa crate cannot run here).

GPU: per-record codes of the batch kernel equal the fixture codes through the
host-buffer, device-resident and verify_rsa entry points."""
import json
import os
import random

import numpy as np
import pytest

from oracle import rsa_oracle as o

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def rv():
    with open(os.path.join(ROOT, "tests", "golden", "rsa_vectors.json")) as f:
        return json.load(f)


def _key(rv, ki):
    return o.parse_spki(bytes.fromhex(rv["keys"][ki]["spki"]))


def test_oracle_matches_fixtures(rv):
    for c in rv["cases"]:
        n, e = _key(rv, c["key"])
        assert o.verify_code(n, e, bytes.fromhex(c["msg"]), bytes.fromhex(c["sig"])) == c["code"], c["name"]
    for b in rv["bad_keys"]:
        with pytest.raises(o.KeyError_):
            o.parse_spki(bytes.fromhex(b["der"]))


def test_reference_round_trip():
    """enclave-verify/src/lib.rs:242-255 with a fixed-seed key."""
    n, e, d = o.gen_key(1024, 65537, random.Random(7))
    doc = o.encode_spki(n, e)
    sig = o.sign_raw(n, d, b"hello world!")
    assert o.verify_rsa(doc, b"hello world!", sig) is True
    assert o.verify_rsa(doc, b"hello world?", sig) is False
    assert o.parse_pkcs1(o.encode_pkcs1(n, e)) == (n, e)


def test_host_der_parser_matches_oracle(rv):
    from cess_amd import bls
    for k in rv["keys"]:
        n, e = o.parse_spki(bytes.fromhex(k["spki"]))
        mod, ee = bls.rsa_parse_key(bytes.fromhex(k["spki"]), bls.RSA_KEY_SPKI)
        assert int.from_bytes(mod, "big") == n and ee == e
        mod, ee = bls.rsa_parse_key(bytes.fromhex(k["pkcs1"]), bls.RSA_KEY_PKCS1)
        assert int.from_bytes(mod, "big") == n and ee == e
    assert len(bytes.fromhex(rv["keys"][0]["pkcs1"])) == 270          # Podr2Key = [u8; 270]
    for b in rv["bad_keys"]:
        with pytest.raises(bls.BlsInfraError) as ei:
            bls.rsa_parse_key(bytes.fromhex(b["der"]), bls.RSA_KEY_SPKI)
        assert ei.value.status == bls.E_BAD_KEY, b["name"]
    # keys the rsa crate accepts but Montgomery arithmetic cannot verify parse
    # like the oracle (never BAD_KEY where the crate has a verdict)
    for u in rv["unsupported_keys"]:
        n, e = o.parse_spki(bytes.fromhex(u["der"]))
        mod, ee = bls.rsa_parse_key(bytes.fromhex(u["der"]), bls.RSA_KEY_SPKI)
        assert int.from_bytes(mod, "big") == n and ee == e, u["name"]


def test_big_class_montgomery_rows_on_host():
    """The loop-form class's Montgomery product (cess_amd/csrc/rsa_mont.hpp,
    RSA_BIG_ROWS rows per pass as a systolic chain) compiled for the host:
    a b R^-1 mod n, below 2n, 28-bit digits, for moduli of 2049-4096 bits and
    operands up to 2n - 1, with the host's padded limb count (multiple of 8)."""
    import ctypes
    import subprocess
    src = os.path.join(ROOT, "tests", "hostemu", "rsa_mont_emu.cpp")
    lib = os.path.join(ROOT, "tests", "hostemu", "librsa_mont_emu.so")
    hdr = os.path.join(ROOT, "cess_amd", "csrc", "rsa_mont.hpp")
    if not os.path.exists(lib) or os.path.getmtime(lib) < max(os.path.getmtime(src), os.path.getmtime(hdr)):
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-DCESS_HOSTEMU", "-shared", "-fPIC", src, "-o", lib])
    emu = ctypes.CDLL(lib)
    M = (1 << 28) - 1
    rng = random.Random(0x4d4f4e54)
    for trial in range(200):
        bits = rng.choice([2049, 2071, 2500, 3001, 3072, 4095, 4096])
        n = rng.getrandbits(bits) | (1 << (bits - 1)) | 1
        kb = (bits + 7) // 8
        L = ((8 * kb + 2 + 27) // 28 + 7) // 8 * 8        # host_rsa.cpp size_class_limbs
        ninv = (-pow(n, -1, 1 << 28)) % (1 << 28)
        a, b = (2 * n - 1, 2 * n - 1) if trial % 10 == 0 else (rng.randrange(2 * n), rng.randrange(2 * n))
        arr = lambda v: (ctypes.c_uint32 * (L + 1))(*[(v >> (28 * i)) & M for i in range(L)] + [0])
        out = (ctypes.c_uint32 * (L + 1))()
        emu.emu_rsa_mont(arr(a), arr(b), arr(n), ctypes.c_uint32(ninv), L, out)
        got = sum(out[i] << (28 * i) for i in range(L + 1))
        assert all(out[i] <= M for i in range(L + 1)), (trial, bits)
        assert got < 2 * n and got % n == a * b * pow(1 << (28 * L), -1, n) % n, (trial, bits)


def _gpu_ctx():
    from cess_amd import bls
    return bls.Context(max_batch=4096)


@pytest.mark.gpu
def test_gpu_fixture_codes(rv):
    from cess_amd import bls
    c = _gpu_ctx()
    try:
        st = c.rsa_keys_load([bytes.fromhex(k["spki"]) for k in rv["keys"]])
        # every size the crate accepts loads: 1024 / 2048-bit classes and the
        # loop-form class (2071, 3001, 3072, 4096 bits)
        assert st == [0] * len(rv["keys"])
        cases = rv["cases"]
        codes = c.rsa_verify_batch([x["key"] for x in cases], [bytes.fromhex(x["msg"]) for x in cases],
                                   [bytes.fromhex(x["sig"]) for x in cases])
        for x, got in zip(cases, codes):
            assert got == x["code"], x["name"]
        assert any(k["bits"] > 2048 for k in rv["keys"]) and any(k["bits"] == 4096 for k in rv["keys"])
        # the PKCS#1 (Podr2Key) encoding gives the same table
        assert c.rsa_keys_load([bytes.fromhex(k["pkcs1"]) for k in rv["keys"]], bls.RSA_KEY_PKCS1) == \
            [0] * len(rv["keys"])
        assert c.rsa_verify_batch([x["key"] for x in cases], [bytes.fromhex(x["msg"]) for x in cases],
                                  [bytes.fromhex(x["sig"]) for x in cases]) == bytes(x["code"] for x in cases)
        # out-of-range key index -> KEY
        assert c.rsa_verify_batch([len(rv["keys"])], [b"x"], [bytes(256)]) == bytes([5])
    finally:
        c.close()


@pytest.mark.gpu
def test_gpu_verify_rsa_dropin(rv):
    from cess_amd import bls
    c = _gpu_ctx()
    try:
        for x in rv["cases"]:
            k = rv["keys"][x["key"]]
            der, msg, sig = bytes.fromhex(k["spki"]), bytes.fromhex(x["msg"]), bytes.fromhex(x["sig"])
            assert c.verify_rsa(der, msg, sig) == (x["code"] == 0), x["name"]   # every size: a verdict
        for b in rv["bad_keys"]:
            with pytest.raises(bls.BlsInfraError) as ei:
                c.verify_rsa(bytes.fromhex(b["der"]), b"hello world!", bytes(256))
            assert ei.value.status == bls.E_BAD_KEY
        # parsed by the reference, not verifiable here: UNSUPPORTED (the caller's
        # CPU path decides), never BAD_KEY
        for u in rv["unsupported_keys"]:
            with pytest.raises(bls.BlsInfraError) as ei:
                c.verify_rsa(bytes.fromhex(u["der"]), b"hello world!", bytes(256))
            assert ei.value.status == bls.RSA_E_UNSUPPORTED, u["name"]
        st = c.rsa_keys_load([bytes.fromhex(u["der"]) for u in rv["unsupported_keys"]])
        assert st == [bls.RSA_E_UNSUPPORTED] * len(rv["unsupported_keys"])
    finally:
        c.close()


@pytest.mark.gpu
def test_gpu_mixed_sizes_device_batch(rv):
    """Records of all size classes interleaved in one batch (the classify
    kernel's three lists): codes equal the oracle's, including bit flips and
    wrong lengths under the 2049-4096-bit keys."""
    from cess_amd import bls
    rng = random.Random(12)
    parsed = [o.parse_spki(bytes.fromhex(k["spki"])) for k in rv["keys"]]
    recs = []
    for _ in range(600):
        x = rng.choice(rv["cases"])
        msg, sig = bytes.fromhex(x["msg"]), bytes.fromhex(x["sig"])
        if rng.random() < 0.3 and sig:
            sig = sig[:-1] + bytes([sig[-1] ^ rng.randrange(1, 256)])
        n, e = parsed[x["key"]]
        recs.append((x["key"], msg, sig, o.verify_code(n, e, msg, sig)))
    c = _gpu_ctx()
    try:
        assert c.rsa_keys_load([bytes.fromhex(k["spki"]) for k in rv["keys"]]) == [0] * len(rv["keys"])
        got = c.rsa_verify_batch([r[0] for r in recs], [r[1] for r in recs], [r[2] for r in recs])
    finally:
        c.close()
    assert list(got) == [r[3] for r in recs]
    big = [g for r, g in zip(recs, got) if rv["keys"][r[0]]["bits"] > 2048]
    assert {0, 4} <= set(big)


@pytest.mark.gpu
@pytest.mark.parametrize("extra_keys", [0, 20])
def test_gpu_device_batch_many(rv, extra_keys):
    """A few thousand records (random valid/invalid mix over the 2048/1024-bit
    keys, incl. wrong lengths) through the device-resident entry point: codes
    equal the oracle's.  extra_keys = 0: few keys, many records each -> the
    key-sorted, wave-padded lists and k_rsa_verify_2048u (host_rsa.cpp
    policy: <= 4096 keys, >= 256 records per key); 20 unused extra keys in the
    table -> the unsorted lists and k_rsa_verify_2048."""
    from cess_amd import bls
    rng = random.Random(11)
    keys = [k for k in rv["keys"] if k["bits"] in (1024, 2048)]      # the expanded classes only
    parsed = [o.parse_spki(bytes.fromhex(k["spki"])) for k in keys]
    base = [x for x in rv["cases"] if rv["keys"][x["key"]]["bits"] in (1024, 2048)]
    kmap = {rv["keys"].index(k): j for j, k in enumerate(keys)}
    recs = []
    for _ in range(3000):
        x = rng.choice(base)
        msg, sig = bytes.fromhex(x["msg"]), bytes.fromhex(x["sig"])
        u = rng.random()
        if u < 0.3 and sig:
            sig = sig[:-1] + bytes([sig[-1] ^ rng.randrange(1, 256)])
        elif u < 0.33:
            sig = sig[1:]                      # SIG_LEN
        elif u < 0.36:
            msg = bytes(len(sig) - 10)         # MSG_LEN
        kj = kmap[x["key"]]
        n, e = parsed[kj]
        recs.append((kj, msg, sig, o.verify_code(n, e, msg, sig)))
    c = _gpu_ctx()
    try:
        c.rsa_keys_load([bytes.fromhex(k["spki"]) for k in keys] + [bytes.fromhex(keys[0]["spki"])] * extra_keys)
        S = b"".join(r[2] for r in recs)
        M = b"".join(r[1] for r in recs)
        so = np.cumsum([0] + [len(r[2]) for r in recs]).astype(np.uint64)
        mo = np.cumsum([0] + [len(r[1]) for r in recs]).astype(np.uint64)
        d = [c.to_device(np.array([r[0] for r in recs], dtype=np.uint32)), c.to_device(S), c.to_device(so),
             c.to_device(M if M else b"\0"), c.to_device(mo)]
        dc = c.device_alloc(len(recs))
        c.rsa_verify_batch_device(len(recs), d[0], d[1], d[2], d[3], d[4], dc)
        c.synchronize()
        got = c.from_device(dc, len(recs))
        for p in d + [dc]:
            c.device_free(p)
    finally:
        c.close()
    assert list(got) == [r[3] for r in recs]
    assert {0, 1, 3, 4} <= set(got)
