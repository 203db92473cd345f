"""Node-side services of the C ABI: the bounded
verdict cache behind the node host function / batcher
(utils/cess-gpu-verify-runtime), and the decode-only deserialize batch behind
the crate's PublicKey::deserialize / Signature::deserialize
(utils/verify-bls-signatures/src/lib.rs:68-82, :138-152).

CPU (no GPU needed): the cache key derivation (SHA-256) against hashlib; hit,
miss, dedup, FIFO eviction and "unavailable" semantics with no context --
records without a cached verdict are CODE_UNAVAILABLE and nothing is cached,
so the caller's own path decides.
GPU: the cache's one-batch verification of the misses equals the golden codes
(all fixed-length and wrong-length cases), a second call is served from the
cache, and deserialize codes equal the oracle's decode of every golden encoding.
"""
import hashlib
import random

import pytest

from cess_amd import bls


def test_sha256_matches_hashlib():
    rng = random.Random(3)
    for n in (0, 1, 55, 56, 63, 64, 65, 119, 120, 1000):
        d = rng.randbytes(n)
        assert bls.sha256(d) == hashlib.sha256(d).digest()


def _recs(k, seed=1):
    rng = random.Random(seed)
    return [(rng.randbytes(48), rng.randbytes(32), rng.randbytes(96)) for _ in range(k)]


def test_cache_without_device_reports_unavailable():
    c = bls.VerdictCache(16)
    recs = _recs(5)
    st, codes, stats = c.verify(recs, ctx=None)
    assert st == bls.E_NO_DEVICE
    assert codes == bytes([bls.CODE_UNAVAILABLE]) * 5
    assert len(c) == 0 and stats["hits"] == 0          # nothing invented, nothing cached


def test_cache_hits_dedup_and_fifo_eviction():
    c = bls.VerdictCache(4)
    recs = _recs(6, seed=2)
    c.insert(recs[:3], bytes([0, 5, 2]))
    st, codes, stats = c.verify(recs[:3] + [recs[1]], ctx=None)
    assert st == 0 and codes == bytes([0, 5, 2, 5]) and stats["hits"] == 4
    # lengths are part of the key: the same bytes split differently never hit
    s, m, k = recs[0]
    st, codes, _ = c.verify([(s + m[:1], m[1:], k)], ctx=None)
    assert codes == bytes([bls.CODE_UNAVAILABLE])
    # a miss repeated in one call is one record; still unavailable without a context
    st, codes, stats = c.verify([recs[4], recs[4], recs[0]], ctx=None)
    assert st == bls.E_NO_DEVICE and codes == bytes([bls.CODE_UNAVAILABLE] * 2 + [0]) and stats["hits"] == 1
    # capacity 4: inserting 3 more evicts the oldest two (FIFO), memory stays bounded
    c.insert(recs[3:6], bytes([0, 0, 4]))
    assert len(c) == 4
    _, codes, _ = c.verify(recs, ctx=None)
    assert codes == bytes([bls.CODE_UNAVAILABLE, bls.CODE_UNAVAILABLE, 2, 0, 0, 4])
    # refreshing an existing record does not grow the cache
    c.insert([recs[2]], bytes([2]))
    assert len(c) == 4
    with pytest.raises(bls.BlsInfraError):
        c.insert([recs[0]], bytes([bls.CODE_UNAVAILABLE]))   # only verdicts are stored
    c.clear()
    assert len(c) == 0


def test_cache_rejects_null_data_with_nonempty_records():
    """A null record buffer is accepted only when all its records are empty
    (the C ABI reads nothing then); otherwise INVALID_ARG, not a crash."""
    import ctypes
    lib = bls.load_library()
    c = bls.VerdictCache(4)
    u64 = ctypes.c_uint64 * 2
    sig = (ctypes.c_uint8 * 48)()
    pk = (ctypes.c_uint8 * 96)()
    codes = (ctypes.c_uint8 * 1)(0)
    for so, sd, po, pd, mo in ((u64(0, 48), None, u64(0, 96), pk, u64(0, 0)),      # sigs null, 48 bytes claimed
                               (u64(0, 48), sig, u64(0, 96), None, u64(0, 0)),      # keys null
                               (u64(0, 48), sig, u64(0, 96), pk, u64(0, 32))):      # msgs null, 32 bytes claimed
        st = lib.cess_bls_cache_verify_var(c._h, None, 1, sd, so, pd, po, None, mo, codes, None)
        assert st == bls.E_INVALID_ARG
        st = lib.cess_bls_cache_insert_var(c._h, 1, sd, so, pd, po, None, mo, codes)
        assert st == bls.E_INVALID_ARG
    # empty messages with a null message buffer are fine (no device: unavailable)
    st = lib.cess_bls_cache_verify_var(c._h, None, 1, sig, u64(0, 48), pk, u64(0, 96), None, u64(0, 0), codes, None)
    assert st == bls.E_NO_DEVICE and codes[0] == bls.CODE_UNAVAILABLE


def _golden_records(vectors):
    cases = vectors["cases"] + vectors["length_cases"]
    return [(bytes.fromhex(c["sig"]), bytes.fromhex(c["msg"]), bytes.fromhex(c["pk"])) for c in cases], \
        bytes(c["code"] for c in cases)


@pytest.mark.gpu
def test_cache_verify_equals_golden(ctx, vectors):
    recs, expect = _golden_records(vectors)
    c = bls.VerdictCache(1 << 16)
    st, codes, stats = c.verify(recs + recs[:5], ctx=ctx)      # duplicates verified once
    assert st == 0
    assert codes == expect + expect[:5]
    assert stats["verified"] == len(set(recs)) and stats["hits"] == 0
    st, codes, stats = c.verify(recs, ctx=ctx)                  # all served by the cache
    assert st == 0 and codes == expect and stats["hits"] == len(recs) and stats["verified"] == 0


@pytest.mark.gpu
def test_deserialize_equals_oracle(ctx, vectors):
    import oracle.bls_oracle as o

    def code_of(fn, b, n, bad_len, bad_point):
        if len(b) != n:
            return bad_len
        try:
            fn(b)
            return 0
        except o.Invalid:
            return bad_point

    cases = vectors["cases"] + vectors["length_cases"]
    sigs = [bytes.fromhex(c["sig"]) for c in cases]
    pks = [bytes.fromhex(c["pk"]) for c in cases]
    want_s = bytes(code_of(o.g1_from_compressed, s, 48, 1, 2) for s in sigs)
    want_p = bytes(code_of(o.g2_from_compressed, p, 96, 3, 4) for p in pks)
    assert set(want_s) >= {0, 1, 2} and set(want_p) >= {0, 3, 4}
    assert ctx.deserialize_codes(bls.KIND_SIG, sigs) == want_s
    assert ctx.deserialize_codes(bls.KIND_PK, pks) == want_p
    # the reference-API mirror now takes the decode-only path
    ok_pk = next(p for p, w in zip(pks, want_p) if w == 0)
    assert bls.PublicKey.deserialize(ok_pk).serialize() == ok_pk


def _runtime_verify_bls_signature(code, reference_fallback):
    """Python mirror of utils/cess-gpu-verify-runtime runtime::verify_bls_signature
    (what the patched audit extrinsic calls): codes 0-5 are the reference's own
    verdicts, only UNAVAILABLE runs the reference function in wasm."""
    if code == bls.CODE_OK:
        return True
    if code in (1, 2, 3, 4, 5):
        return False
    return reference_fallback()


@pytest.mark.gpu
def test_cache_codes_are_verdicts_for_malformed_records(ctx, vectors):
    """the audit wiring must not reach a panicking verifier.
    cess_bls_cache_verify_var answers every malformed golden record (wrong
    length, non-point, non-subgroup, off-curve, flag abuse) with its code 1-4
    -- a verdict -- never CODE_UNAVAILABLE, so a GPU node decides it exactly as
    the reference's total verify_bls_signature (src/lib.rs:243-247) does on a
    wasm node, with no fallback at all."""
    recs, expect = _golden_records(vectors)
    c = bls.VerdictCache(1 << 16)
    st, codes, stats = c.verify(recs, ctx=ctx)
    assert st == 0 and codes == expect
    assert bls.CODE_UNAVAILABLE not in codes
    assert {1, 2, 3, 4} <= set(codes)          # every malformed kind is present
    fallbacks = []
    for code, want in zip(codes, expect):
        ok = _runtime_verify_bls_signature(code, lambda: fallbacks.append(1) or True)
        assert ok == (want == 0)
    assert not fallbacks
