"""Generate tests/golden/rsa_vectors.json from the RSA oracle (oracle/rsa_oracle.py).

Deterministic (seeded) keys of 1024 / 2048 / 2071 / 3001 / 3072 / 4096 bits,
e = 65537 and e = 3,
each as SPKI DER (what cp_enclave_verify::verify_rsa parses) and PKCS#1 DER
(Podr2Key = [u8; 270], primitives/common/src/lib.rs:54), with valid and
invalid raw PKCS#1 v1.5 signatures (Pkcs1v15Sign::new_raw()) -- including the
reference test's own message "hello world!" (enclave-verify/src/lib.rs:248) --
plus malformed DER keys.  Parity is UNPINNED (see the oracle's header).

Usage: python tests/golden/gen_rsa.py
"""
import json
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import rsa_oracle as o  # noqa: E402


def main():
    rng = random.Random(0x525341)
    keys = []
    for bits, e in ((2048, 65537), (2048, 65537), (1024, 65537), (3072, 65537), (2048, 3)):
        n, e, d = o.gen_key(bits, e, rng)
        keys.append({"n": n, "e": e, "d": d})
    out_keys = [{"bits": k["n"].bit_length(), "e": k["e"], "spki": o.encode_spki(k["n"], k["e"]).hex(),
                 "pkcs1": o.encode_pkcs1(k["n"], k["e"]).hex()} for k in keys]
    cases = []

    def add(name, ki, msg, sig):
        k = keys[ki]
        cases.append({"name": name, "key": ki, "msg": msg.hex(), "sig": sig.hex(),
                      "code": o.verify_code(k["n"], k["e"], msg, sig)})

    for ki, k in enumerate(keys):
        n, d = k["n"], k["d"]
        kb = (n.bit_length() + 7) // 8
        hw = b"hello world!"                                 # the reference test's message
        add(f"k{ki}_hello_world", ki, hw, o.sign_raw(n, d, hw))
        for j in range(3):
            m = bytes(rng.randrange(256) for _ in range(32))
            add(f"k{ki}_valid32_{j}", ki, m, o.sign_raw(n, d, m))
        add(f"k{ki}_empty_msg", ki, b"", o.sign_raw(n, d, b""))
        mx = bytes(rng.randrange(256) for _ in range(kb - 11))
        add(f"k{ki}_max_msg", ki, mx, o.sign_raw(n, d, mx))
        s = o.sign_raw(n, d, hw)
        add(f"k{ki}_wrong_msg", ki, b"hello world?", s)
        add(f"k{ki}_flipped_sig", ki, hw, s[:-1] + bytes([s[-1] ^ 1]))
        add(f"k{ki}_short_sig", ki, hw, s[1:])
        add(f"k{ki}_long_sig", ki, hw, b"\x00" + s)
        add(f"k{ki}_sig_eq_n", ki, hw, n.to_bytes(kb, "big"))
        add(f"k{ki}_sig_max", ki, hw, b"\xff" * kb)
        add(f"k{ki}_sig_zero", ki, hw, bytes(kb))
        add(f"k{ki}_sig_one", ki, b"", (1).to_bytes(kb, "big"))
        add(f"k{ki}_msg_too_long", ki, bytes(kb - 10), s)
        add(f"k{ki}_msg_too_long_sig_max", ki, bytes(kb - 10), b"\xff" * kb)   # length code first
        # wrong block type (0x02) and a missing separator, both validly exponentiated
        for nm, em in (("bt02", b"\x00\x02" + b"\xff" * (kb - len(hw) - 3) + b"\x00" + hw),
                       ("nosep", b"\x00\x01" + b"\xff" * (kb - len(hw) - 2) + hw),
                       ("short_ps", b"\x00\x01" + b"\xff" * 7 + b"\x00" + bytes(kb - 10))):
            add(f"k{ki}_{nm}", ki, hw if nm != "short_ps" else bytes(kb - 10),
                pow(int.from_bytes(em, "big"), d, n).to_bytes(kb, "big"))
    # malformed keys (verify_rsa panics: PublicKey::from_public_key_der(..).unwrap())
    good = bytes.fromhex(out_keys[0]["spki"])
    bad_keys = [{"name": "truncated", "der": good[:-1].hex()},
                {"name": "trailing", "der": (good + b"\x00").hex()},
                {"name": "wrong_oid", "der": good.replace(o.RSA_OID, bytes.fromhex("2a8648ce3d0201")).hex()},
                {"name": "pkcs1_not_spki", "der": out_keys[0]["pkcs1"]},
                {"name": "e_one", "der": o.encode_spki(keys[0]["n"], 1).hex()},
                {"name": "empty", "der": ""}]
    for b in bad_keys:
        try:
            o.parse_spki(bytes.fromhex(b["der"]))
            b["parses"] = True
        except o.KeyError_:
            b["parses"] = False
    assert not any(b["parses"] for b in bad_keys)
    # keys the rsa crate parses (check_public has no parity check; the SPKI
    # parameters are not inspected) but Montgomery arithmetic cannot verify:
    # the GPU library reports CESS_RSA_E_UNSUPPORTED for them, never BAD_KEY
    alg_params = (b"\x30\x0d\x06\x09" + o.RSA_OID + b"\x05\x00",
                  b"\x30\x0f\x06\x09" + o.RSA_OID + b"\x04\x02\xab\xcd")
    unsupported = [{"name": "even_modulus", "der": o.encode_spki(keys[0]["n"] + 1, 65537).hex()},
                   {"name": "modulus_one", "der": o.encode_spki(1, 65537).hex()},
                   {"name": "params_not_null", "der": good.replace(alg_params[0], alg_params[1])
                    .replace(good[:4], good[:3] + bytes([good[3] + 2])).hex()}]
    for u in unsupported:
        n_, e_ = o.parse_spki(bytes.fromhex(u["der"]))     # parses (the reference accepts it)
        u["n_bits"] = n_.bit_length()
    # bench pool (bench.py --mode rsa): valid raw signatures over 32-byte
    # messages under key 0 (2048-bit), replicated by the bench to its batch size
    n0, d0 = keys[0]["n"], keys[0]["d"]
    pool = []
    for _ in range(256):
        m = bytes(rng.randrange(256) for _ in range(32))
        pool.append({"msg": m.hex(), "sig": o.sign_raw(n0, d0, m).hex()})
    # moduli of the loop-form GPU class (2049-4096 bits, k_rsa_verify_big):
    # 4096 bits (the crate's maximum), 2071 bits (the smallest size above the
    # 2048-bit class, 75 limbs) and 3001 bits with e = 3, from their own seed
    # so the vectors above stay as they were
    rng2 = random.Random(0x52534132)
    for bits, e in ((4096, 65537), (2071, 65537), (3001, 3)):
        n, e, d = o.gen_key(bits, e, rng2)
        keys.append({"n": n, "e": e, "d": d})
        out_keys.append({"bits": n.bit_length(), "e": e, "spki": o.encode_spki(n, e).hex(),
                         "pkcs1": o.encode_pkcs1(n, e).hex()})
        ki = len(keys) - 1
        kb = (n.bit_length() + 7) // 8
        hw = b"hello world!"
        s = o.sign_raw(n, d, hw)
        add(f"k{ki}_hello_world", ki, hw, s)
        for j in range(2):
            m = bytes(rng2.randrange(256) for _ in range(32))
            add(f"k{ki}_valid32_{j}", ki, m, o.sign_raw(n, d, m))
        mx = bytes(rng2.randrange(256) for _ in range(kb - 11))
        add(f"k{ki}_max_msg", ki, mx, o.sign_raw(n, d, mx))
        add(f"k{ki}_empty_msg", ki, b"", o.sign_raw(n, d, b""))
        add(f"k{ki}_wrong_msg", ki, b"hello world?", s)
        add(f"k{ki}_flipped_sig", ki, hw, s[:-1] + bytes([s[-1] ^ 1]))
        add(f"k{ki}_short_sig", ki, hw, s[1:])
        add(f"k{ki}_sig_eq_n", ki, hw, n.to_bytes(kb, "big"))
        add(f"k{ki}_sig_max", ki, hw, b"\xff" * kb)
        add(f"k{ki}_sig_one", ki, b"", (1).to_bytes(kb, "big"))
        add(f"k{ki}_msg_too_long", ki, bytes(kb - 10), s)
        em = b"\x00\x02" + b"\xff" * (kb - len(hw) - 3) + b"\x00" + hw
        add(f"k{ki}_bt02", ki, hw, pow(int.from_bytes(em, "big"), d, n).to_bytes(kb, "big"))
    # moduli just above the 1024-bit class's limb span (37 x 28 = 1036 bits):
    # 1033 / 1034-bit keys have k = 130-byte signatures (1040 bits), so a
    # signature s + 2^1036 (>= n: SIG_RANGE) differs from a valid s only in bits
    # the 1024-bit class has no limb for -- the host must route these keys to a
    # class whose limbs cover all 8 k signature bits.  1032 bits (k = 129) is
    # the largest key that stays in the 1024-bit class.  Own seed.
    rng3 = random.Random(0x52534133)
    for bits in (1033, 1034, 1032):
        n, e, d = o.gen_key(bits, 65537, rng3)
        keys.append({"n": n, "e": e, "d": d})
        out_keys.append({"bits": n.bit_length(), "e": e, "spki": o.encode_spki(n, e).hex(),
                         "pkcs1": o.encode_pkcs1(n, e).hex()})
        ki = len(keys) - 1
        kb = (n.bit_length() + 7) // 8
        hw = b"hello world!"
        s = o.sign_raw(n, d, hw)
        add(f"k{ki}_hello_world", ki, hw, s)
        m = bytes(rng3.randrange(256) for _ in range(32))
        add(f"k{ki}_valid32", ki, m, o.sign_raw(n, d, m))
        si = int.from_bytes(s, "big")
        for top in (1036, 1037, 1039):
            if si + (1 << top) < (1 << (8 * kb)):
                add(f"k{ki}_sig_plus_2^{top}", ki, hw, (si + (1 << top)).to_bytes(kb, "big"))
        add(f"k{ki}_sig_top_bit", ki, hw, (si | (1 << (8 * kb - 1))).to_bytes(kb, "big"))
        add(f"k{ki}_sig_eq_n", ki, hw, n.to_bytes(kb, "big"))
        add(f"k{ki}_sig_max", ki, hw, b"\xff" * kb)
        add(f"k{ki}_flipped_sig", ki, hw, s[:-1] + bytes([s[-1] ^ 1]))
    doc = {"generator": "tests/golden/gen_rsa.py (oracle/rsa_oracle.py)",
           "codes": {"0": "OK", "1": "SIG_LEN", "2": "SIG_RANGE", "3": "MSG_LEN", "4": "MISMATCH"},
           "keys": out_keys, "cases": cases, "bad_keys": bad_keys,
           "unsupported_keys": unsupported, "bench_pool_key0": pool}
    with open(os.path.join(ROOT, "tests", "golden", "rsa_vectors.json"), "w") as f:
        json.dump(doc, f, indent=1)
    print(len(cases), "cases,", len(bad_keys), "bad keys")


if __name__ == "__main__":
    main()
