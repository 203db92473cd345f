"""GPU: edge cases of the batch boundary -- partial bitmap words, empty
batches, the device-resident entry point against the host one, the adversarial
mix of BASELINE config[4] at moderate size (codes exact against the oracle's
fixture codes), and identity keys in RLC mode."""
import json
import os
import random

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001


def _signed(ctx, n, seed, msg_len=32):
    rng = random.Random(seed)
    sks = [rng.randrange(1, R).to_bytes(32, "big") for _ in range(n)]
    msgs = [rng.randbytes(msg_len) for _ in range(n)]
    return ctx.sign(sks, msgs), msgs, ctx.public_keys(sks)


def _offs(msgs):
    o = [0]
    for m in msgs:
        o.append(o[-1] + len(m))
    return o


@pytest.mark.parametrize("n", [1, 63, 65, 130])
def test_partial_bitmap_words(ctx, n):
    sigs, msgs, pks = _signed(ctx, n, n)
    msgs[-1] = bytes(len(msgs[-1]))           # last record forged
    codes, words = ctx.verify_fixed(b"".join(sigs), b"".join(pks), b"".join(msgs), _offs(msgs))
    assert list(codes) == [0] * (n - 1) + [5]
    assert len(words) == (n + 63) // 64
    bits = [(words[i >> 6] >> (i & 63)) & 1 for i in range(n)]
    assert bits == [1] * (n - 1) + [0]
    if n % 64:
        assert words[-1] >> (n % 64) == 0      # no bits set past the last record


def test_empty_batch(ctx):
    assert ctx.verify_codes([]) == b""
    codes, words = ctx.verify_fixed(b"", b"", b"", [0])
    assert codes == b"" and words == []


def test_var_batch_null_buffers(ctx):
    """cess_bls_verify_batch_var: a null signature / key buffer is accepted only
    when every record of it is empty (all WrongLength); otherwise INVALID_ARG."""
    import ctypes
    from cess_amd import bls
    lib = ctx._lib
    u64 = ctypes.c_uint64 * 2
    codes = (ctypes.c_uint8 * 1)()
    pk = (ctypes.c_uint8 * 96)()
    sig = (ctypes.c_uint8 * 48)()
    st = lib.cess_bls_verify_batch_var(ctx._h, 1, None, u64(0, 48), pk, u64(0, 96), None, u64(0, 0), codes, None)
    assert st == bls.E_INVALID_ARG
    st = lib.cess_bls_verify_batch_var(ctx._h, 1, sig, u64(0, 48), None, u64(0, 96), None, u64(0, 0), codes, None)
    assert st == bls.E_INVALID_ARG
    st = lib.cess_bls_verify_batch_var(ctx._h, 1, None, u64(0, 0), pk, u64(0, 96), None, u64(0, 0), codes, None)
    assert st == 0 and codes[0] == 1             # empty signature: SIG_LEN, nothing read


def _hip():
    """The HIP runtime libcess_bls.so itself links (/opt/rocm), via ctypes, so
    device buffers come from the same runtime instance as the kernels (torch
    bundles a second HIP runtime; initialising both in one process is
    order-sensitive)."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    hip.hipFree.argtypes = [ctypes.c_void_p]
    hip.hipDeviceSynchronize.argtypes = []
    return hip


def test_device_entry_matches_host(ctx):
    import ctypes
    hip = _hip()
    n = 256
    sigs, msgs, pks = _signed(ctx, n, 11)
    msgs[7] = bytes(32)
    S, P, M = b"".join(sigs), b"".join(pks), b"".join(msgs)
    expect, ewords = ctx.verify_fixed(S, P, M, _offs(msgs))
    offs = (ctypes.c_uint64 * (n + 1))(*_offs(msgs))
    ptrs = []

    def dev(data, size):
        p = ctypes.c_void_p()
        assert hip.hipMalloc(ctypes.byref(p), size) == 0
        if data is not None:
            assert hip.hipMemcpy(p, data, size, 1) == 0          # host -> device
        ptrs.append(p)
        return p.value

    try:
        d_s, d_p, d_m = dev(S, len(S)), dev(P, len(P)), dev(M, len(M))
        d_o = dev(ctypes.cast(offs, ctypes.c_void_p), 8 * (n + 1))
        d_c, d_b = dev(None, n), dev(None, 8 * (n // 64))
        ctx.verify_device(n, d_s, d_p, d_m, d_o, d_c, d_b)
        assert hip.hipDeviceSynchronize() == 0
        codes = (ctypes.c_uint8 * n)()
        words = (ctypes.c_uint64 * (n // 64))()
        assert hip.hipMemcpy(codes, ctypes.c_void_p(d_c), n, 2) == 0   # device -> host
        assert hip.hipMemcpy(words, ctypes.c_void_p(d_b), 8 * (n // 64), 2) == 0
    finally:
        for p in ptrs:
            hip.hipFree(p)
    assert bytes(codes) == expect
    assert list(words) == ewords


def test_adversarial_mix_exact_codes(ctx, vectors):
    """config[4] shape at 20,000 records: 1 % forged, 1 % adversarial fixture
    records (non-subgroup, off-curve, x >= p, flag errors, identities) through
    both the fixed-stride and the variable-length entry points."""
    n = 20000
    sigs, msgs, pks = _signed(ctx, n, 12)
    rng = random.Random(13)
    expect = [0] * n
    cases = [c for c in vectors["cases"] if len(c["sig"]) == 96 and len(c["pk"]) == 192]
    idx = rng.sample(range(n), 400)
    for i in idx[:200]:
        msgs[i] = rng.randbytes(32)
        expect[i] = 5
    for j, i in enumerate(idx[200:]):
        c = cases[j % len(cases)]
        sigs[i], msgs[i], pks[i] = bytes.fromhex(c["sig"]), bytes.fromhex(c["msg"]), bytes.fromhex(c["pk"])
        expect[i] = c["code"]
    codes, _ = ctx.verify_fixed(b"".join(sigs), b"".join(pks), b"".join(msgs), _offs(msgs))
    assert list(codes) == expect
    # variable-length path, with the golden wrong-length records appended
    lc = vectors["length_cases"]
    recs = list(zip(sigs, msgs, pks)) + [(bytes.fromhex(c["sig"]), bytes.fromhex(c["msg"]), bytes.fromhex(c["pk"]))
                                         for c in lc]
    assert list(ctx.verify_codes(recs)) == expect + [c["code"] for c in lc]


def test_rlc_identity_keys(ctx, vectors):
    """RLC groups by key encoding: the identity key (its pairing term is 1) and
    the (O, O) pair must come out exactly as in the per-signature path."""
    sigs, msgs, pks = _signed(ctx, 3000, 14)
    ident = next(c for c in vectors["cases"] if c["sig"].startswith("c0") and c["pk"].startswith("c0"))
    O_sig, O_pk = bytes.fromhex(ident["sig"]), bytes.fromhex(ident["pk"])
    for i in (5, 700, 2999):
        sigs[i], pks[i] = O_sig, O_pk                 # (O, O): accepted for any message
    pks[1000] = O_pk                                  # valid sig, identity key: rejected
    S, P, M, o = b"".join(sigs), b"".join(pks), b"".join(msgs), _offs(msgs)
    expect, _ = ctx.verify_fixed(S, P, M, o)
    codes, _, st = ctx.verify_rlc(S, P, M, o, seed=bytes(range(32)))
    assert codes == expect
    assert expect[5] == expect[700] == 0 and expect[1000] == 5
    assert json.dumps(st)


def test_g2_subgroup_check_on_prepared_point(ctx):
    """k_decode_pk decodes keys on-curve only; k_prepare rejects a key whose
    psi(Q) != -[|x|]Q on the T of its G2Prepared iteration.  Random on-curve
    G2 points outside the subgroup (cofactor not cleared, oracle-encoded) must
    come back PK_POINT (4) -- per record and in the keyed batch's key table --
    while a bad signature's code keeps precedence over the key's and the
    valid records around them stay 0 (codes equal the oracle's)."""
    import oracle.bls_oracle as o
    rng = random.Random(41)
    bad = []
    while len(bad) < 6:
        x = (rng.randrange(o.P), rng.randrange(o.P))
        rhs = o.f2_add(o.f2_mul(o.f2_sqr(x), x), (4, 4))
        if not o.f2_is_square(rhs):
            continue
        pt = (x, o.f2_sqrt(rhs))
        if not o.g2_in_subgroup(pt):
            bad.append(o.g2_to_compressed(pt))
    sigs, msgs, pks = _signed(ctx, 16, 7)
    recs = list(zip(sigs, msgs, pks))
    for j, k in enumerate(bad):
        recs[2 * j + 1] = (recs[2 * j + 1][0], recs[2 * j + 1][1], k)
    recs[3] = (recs[3][0][:-1] + bytes([recs[3][0][-1] ^ 1]), recs[3][1], recs[3][2])   # bad sig + bad key
    want = [o.verify_code(*r) for r in recs]
    assert want.count(4) == 5 and want[3] in (1, 2)
    assert list(ctx.verify_codes(recs)) == want
    # distinct-key table: one bad key among good ones
    keys = [pks[0], bad[0], pks[2]]
    kc = ctx.load_keys(keys)
    assert list(kc) == [0, 4, 0]
