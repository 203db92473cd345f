"""Generate tests/golden/vectors.json from the CPU oracle (oracle/bls_oracle.py).

The vectors are DATA: inputs + expected outputs.  They cover
  * every known-answer test of the reference crate
    (utils/verify-bls-signatures/tests/tests.rs:19-112), verbatim,
  * seeded random valid signatures (various message lengths, incl. empty),
  * forged signatures (valid points, wrong message),
  * malformed / adversarial encodings (SURVEY §8(d) C5 list): G1/G2 points off
    the subgroup, off the curve, x >= p, compression bit clear, infinity flag
    with x != 0, infinity + sort flag, identity encodings, (O, O) pairs,
    wrong lengths,
  * Gt bytes of the pairing product for valid and forged records (parity
    unpinned by the reference; pinned against this oracle),
  * hash_to_g1 outputs and keygen/sign vectors.
Run:  python tests/golden/gen_golden.py
"""
import json
import os
import random
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import oracle.bls_oracle as o  # noqa: E402

KAT_SRC = "utils/verify-bls-signatures/tests/tests.rs"
M1 = "0d69632d73746174652d726f6f74e6c01e909b4923345ce5970962bcfe3004bfd8474a21dae28f50692502f46d90"
M2 = "0d69632d73746174652d726f6f74b294b418b11ebe5dd7dd1dcb099e4e0372b9a42aef7a7a37fb4f25667d705ea9"
S1 = "ace9fcdd9bc977e05d6328f889dc4e7c99114c737a494653cb27a1f55c06f4555e0f160980af5ead098acc195010b2f7"
S2 = "89a2be21b5fa8ac9fab1527e041327ce899d7da971436a1f2165393947b4d942365bfe5488710e61a619ba48388a21b1"
K1 = ("814c0e6ec71fab583b08bd81373c255c3c371b2e84863c98a4f1e08b74235d14fb5d9c0cd546d9685f913a0c0b2cc534"
      "1583bf4b4392e467db96d65b9bb4cb717112f8472e0d5a4d14505ffd7484b01291091c5f87b98883463f98091a0baaae")
K2 = ("9933e1f89e8a3c4d7fdcccdbd518089e2bd4d8180a261f18d9c247a52768ebce98dc7328a39814a8f911086a1dd50cbe"
      "015e2a53b7bf78b55288893daa15c346640e8831d72a12bdedd979d28470c34823b8d1c3f4795d9c3984a247132e94fe")
IC_PK = ("87033f48fd8f327ff5d164e85af31433c6a8c73fc5a65bad5d472127205c73c5168a45e862f5af6d0da5676df45d0a5f"
         "1293a530d5498f812a34a280f6bef869e4ca9b7c275554456d8770733d72ac4006777382fa541873fe002adb12184268")
IC_MSG = ("e751fdb69185002b13c8d2954c7d0c39546402ecdde9c2a9a2c624293535a5ca2f560a582f705580448fbe1ccdc0e86af3"
          "ba4c487a7f73bc9c312556")
IC_SIG = "98733cc2b312d5787cd4dba6ea0e19a1f1850b9e8c6d5112f12e12db8e7413a4ecb4096c23730566c67d9b2694e4e179"
SIGN_SK = "6f3977f6051e184b2c412daa1b5c0115ef7ab347cac8d808ffa2c26bd0658243"
SIGN_MSG = ("50484522ad8aede64ec7f86b9273b7ed3940481acf93cdd40a2b77f2be2734a14012b2492b6363b12adaeaf055c573e4611b"
            "085d2e0fe2153d72453a95eaebf350ac3ba6a26ba0bc79f4c0bf5664dfdf5865f69f7fc6b58ba7d068e8")
SIGN_EXP = "8f7ad830632657f7b3eae17fd4c3d9ff5c13365eea8d33fd0a1a6d8fbebc5152e066bb0ad61ab64e8a8541c8e3f96de9"


def flip_last(h, new):
    return h[:-2] + new


def main():
    rng = random.Random(0xC0FFEE)
    cases = []

    def add(name, sig, msg, pk, src=None, expect_ok=None, gt=False):
        sig_b, msg_b, pk_b = bytes.fromhex(sig), bytes.fromhex(msg), bytes.fromhex(pk)
        code = o.verify_code(sig_b, msg_b, pk_b)
        if expect_ok is not None:
            assert (code == 0) == expect_ok, (name, code)
        rec = {"name": name, "sig": sig, "msg": msg, "pk": pk, "code": code}
        if src:
            rec["ref"] = src
        if gt and code in (0, 5):
            s = o.g1_from_compressed(sig_b)
            k = o.g2_from_compressed(pk_b)
            rec["gt"] = o.gt_to_bytes(o.verify_gt(s, msg_b, k)).hex()
        cases.append(rec)

    # --- reference KATs (tests.rs) ---
    add("kat_verify_valid_1", S1, M1, K1, KAT_SRC + ":22-26", True, gt=True)
    add("kat_verify_valid_2", S2, M2, K2, KAT_SRC + ":28-32", True, gt=True)
    add("kat_reject_invalid_1", S2, M1, K1, KAT_SRC + ":38-42", False, gt=True)
    add("kat_reject_invalid_2", S1, M2, K2, KAT_SRC + ":44-48", False, gt=True)
    add("kat_reject_invalid_sig", flip_last(S1, "f8"), M1, K1, KAT_SRC + ":54-58", False)
    add("kat_reject_invalid_key", S1, M1, flip_last(K1, "ad"), KAT_SRC + ":64-68", False)
    add("kat_known_good_ic", IC_SIG, IC_MSG, IC_PK, KAT_SRC + ":88-97", True, gt=True)
    assert cases[4]["code"] == o.SIG_POINT and cases[5]["code"] == o.PK_POINT

    # --- seeded random valid + forged ---
    keys = []
    for i, mlen in enumerate([0, 1, 24, 32, 32, 32, 46, 55, 56, 64, 72, 73, 100, 136, 137, 200]):
        sk = rng.randrange(1, o.R)
        msg = bytes(rng.randrange(256) for _ in range(mlen))
        pk = o.public_key(sk)
        sig = o.sign(sk, msg)
        keys.append((sk, pk, sig, msg))
        add(f"valid_len{mlen}_{i}", sig.hex(), msg.hex(), pk.hex(), expect_ok=True, gt=(i % 4 == 0))
    for i in range(6):
        sk, pk, sig, msg = keys[i + 2]
        msg2 = bytes(rng.randrange(256) for _ in range(32))
        add(f"forged_msg_{i}", sig.hex(), msg2.hex(), pk.hex(), expect_ok=False, gt=(i < 2))
        sk2, pk2, _, _ = keys[i + 8]
        add(f"forged_key_{i}", sig.hex(), msg.hex(), pk2.hex(), expect_ok=False)
    good_sig, good_pk, good_msg = keys[3][2].hex(), keys[3][1].hex(), keys[3][3].hex()

    # --- adversarial encodings ---
    def g1_nonsubgroup():
        while True:
            x = rng.randrange(o.P)
            y = o.fp_sqrt((x ** 3 + 4) % o.P)
            if y is not None and not o.g1_in_subgroup((x, y)):
                return o.g1_to_compressed((x, y))

    def g2_nonsubgroup():
        while True:
            x = (rng.randrange(o.P), rng.randrange(o.P))
            y = o.f2_sqrt(o.f2_add(o.f2_mul(o.f2_sqr(x), x), o.B2))
            if y is not None and not o.g2_in_subgroup((x, y)):
                return o.g2_to_compressed((x, y))

    def g1_offcurve():
        while True:
            x = rng.randrange(o.P)
            if o.fp_sqrt((x ** 3 + 4) % o.P) is None:
                b = bytearray(x.to_bytes(48, "big"))
                b[0] |= 0x80 | (0x20 if rng.random() < 0.5 else 0)
                return bytes(b)

    def g2_offcurve():
        while True:
            x = (rng.randrange(o.P), rng.randrange(o.P))
            if o.f2_sqrt(o.f2_add(o.f2_mul(o.f2_sqr(x), x), o.B2)) is None:
                b = bytearray(x[1].to_bytes(48, "big") + x[0].to_bytes(48, "big"))
                b[0] |= 0x80
                return bytes(b)

    for i in range(3):
        add(f"sig_g1_nonsubgroup_{i}", g1_nonsubgroup().hex(), good_msg, good_pk, expect_ok=False)
        add(f"pk_g2_nonsubgroup_{i}", good_sig, good_msg, g2_nonsubgroup().hex(), expect_ok=False)
        add(f"sig_offcurve_{i}", g1_offcurve().hex(), good_msg, good_pk, expect_ok=False)
        add(f"pk_offcurve_{i}", good_sig, good_msg, g2_offcurve().hex(), expect_ok=False)
    # small-order points: (0, +-2) on G1 has order 3
    add("sig_order3_point", o.g1_to_compressed((0, 2)).hex(), good_msg, good_pk, expect_ok=False)
    # x >= p
    pbytes = bytearray(o.P.to_bytes(48, "big"))
    pbytes[0] |= 0x80
    add("sig_x_eq_p", pbytes.hex(), good_msg, good_pk, expect_ok=False)
    big = bytearray(((1 << 381) - 1).to_bytes(48, "big"))
    big[0] |= 0x80
    add("sig_x_max", big.hex(), good_msg, good_pk, expect_ok=False)
    pk_c1_big = bytearray(bytes.fromhex(good_pk))
    pk_c1_big[0:48] = pbytes
    add("pk_x_c1_eq_p", good_sig, good_msg, bytes(pk_c1_big).hex(), expect_ok=False)
    pk_c0_big = bytearray(bytes.fromhex(good_pk))
    pk_c0_big[48:96] = (o.P + 5).to_bytes(48, "big")
    add("pk_x_c0_gt_p", good_sig, good_msg, bytes(pk_c0_big).hex(), expect_ok=False)
    # flags
    s = bytearray(bytes.fromhex(good_sig))
    s[0] &= 0x7F
    add("sig_compression_bit_clear", bytes(s).hex(), good_msg, good_pk, expect_ok=False)
    s = bytearray(bytes.fromhex(good_sig))
    s[0] |= 0x40
    add("sig_infinity_flag_nonzero_x", bytes(s).hex(), good_msg, good_pk, expect_ok=False)
    k = bytearray(bytes.fromhex(good_pk))
    k[0] &= 0x7F
    add("pk_compression_bit_clear", good_sig, good_msg, bytes(k).hex(), expect_ok=False)
    k = bytearray(bytes.fromhex(good_pk))
    k[0] |= 0x40
    add("pk_infinity_flag_nonzero_x", good_sig, good_msg, bytes(k).hex(), expect_ok=False)
    inf_sig = bytearray(48)
    inf_sig[0] = 0xC0
    inf_pk = bytearray(96)
    inf_pk[0] = 0xC0
    bad_inf_sig = bytearray(inf_sig)
    bad_inf_sig[0] = 0xE0
    add("sig_infinity_plus_sort", bad_inf_sig.hex(), good_msg, good_pk, expect_ok=False)
    bad_inf_pk = bytearray(inf_pk)
    bad_inf_pk[0] = 0xE0
    add("pk_infinity_plus_sort", good_sig, good_msg, bad_inf_pk.hex(), expect_ok=False)
    nocomp_inf = bytearray(48)
    nocomp_inf[0] = 0x40
    add("sig_infinity_without_compression", nocomp_inf.hex(), good_msg, good_pk, expect_ok=False)
    zero_sig = bytearray(48)
    zero_sig[0] = 0x80
    add("sig_x_zero_no_inf_flag", zero_sig.hex(), good_msg, good_pk, expect_ok=False)
    # identity handling (A16): (O, O) verifies for any message; O with a real key does not
    for i, m in enumerate(["", "00", good_msg]):
        add(f"identity_pair_{i}", inf_sig.hex(), m, inf_pk.hex(), expect_ok=True)
    add("identity_sig_real_pk", inf_sig.hex(), good_msg, good_pk, expect_ok=False)
    add("real_sig_identity_pk", good_sig, good_msg, inf_pk.hex(), expect_ok=False)
    # precedence: invalid sig + invalid key -> SIG_POINT
    add("precedence_bad_sig_bad_key", g1_offcurve().hex(), good_msg, g2_offcurve().hex(), expect_ok=False)
    assert cases[-1]["code"] == o.SIG_POINT

    # wrong lengths (variable-length API)
    lens = []

    def addlen(name, sig, msg, pk, code):
        got = o.verify_code(bytes.fromhex(sig), bytes.fromhex(msg), bytes.fromhex(pk))
        assert got == code, (name, got)
        lens.append({"name": name, "sig": sig, "msg": msg, "pk": pk, "code": got})
    addlen("sig_len_47", good_sig[:-2], good_msg, good_pk, o.SIG_LEN)
    addlen("sig_len_49", good_sig + "00", good_msg, good_pk, o.SIG_LEN)
    addlen("sig_len_0", "", good_msg, good_pk, o.SIG_LEN)
    addlen("pk_len_95", good_sig, good_msg, good_pk[:-2], o.PK_LEN)
    addlen("pk_len_97", good_sig, good_msg, good_pk + "00", o.PK_LEN)
    addlen("bad_sig_and_pk_len", g1_offcurve().hex(), good_msg, good_pk[:-2], o.SIG_POINT)
    addlen("sig_len_bad_pk_len_bad", good_sig[:-2], good_msg, good_pk[:-2], o.SIG_LEN)

    # hash_to_g1 and generator vectors
    h2c = []
    for m in [b"", b"abc", bytes(32), bytes(range(100)), bytes(200)]:
        h2c.append({"msg": m.hex(), "h": o.g1_to_compressed(o.hash_to_g1(m)).hex()})
    gen = [{"sk": SIGN_SK, "msg": SIGN_MSG, "sig": SIGN_EXP, "ref": KAT_SRC + ":99-112",
            "pk": o.public_key(int(SIGN_SK, 16))}]
    assert o.sign(int(SIGN_SK, 16), bytes.fromhex(SIGN_MSG)).hex() == SIGN_EXP
    gen[0]["pk"] = gen[0]["pk"].hex()
    for sk, pk, sig, msg in keys[:8]:
        gen.append({"sk": o.sk_serialize(sk).hex(), "msg": msg.hex(), "sig": sig.hex(), "pk": pk.hex()})

    out = {
        "generator": "tests/golden/gen_golden.py (oracle/bls_oracle.py)",
        "codes": {"0": "OK", "1": "SIG_LEN", "2": "SIG_POINT", "3": "PK_LEN", "4": "PK_POINT", "5": "PAIRING_FAIL"},
        "cases": cases, "length_cases": lens, "hash_to_g1": h2c, "keygen_sign": gen,
    }
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "vectors.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(f"wrote {path}: {len(cases)} cases, {len(lens)} length cases")


if __name__ == "__main__":
    main()
