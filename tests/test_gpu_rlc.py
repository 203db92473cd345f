"""GPU: RLC batch mode (random linear combination + bisection, BASELINE config
4 shape: few keys).  Parity bar: the per-record codes equal the per-signature
path's (cess_bls_verify_batch) on the same records, including forged,
malformed, non-subgroup and identity inputs, and the cross-shard Gt-product
combine gives the same verdicts as one shard.  Every test runs with the
first check's sums from the bucket kernels (k_msm_*, env CESS_BLS_RLC_MSM=1)
and from per-record scalar multiples (=0); the Gt value of a failing check is
the same group element either way (test_rlc_bucket_sums_equal_scalar_multiples)."""
import os
import random

import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, params=["msm", "scale"])
def rlc_sums_path(request):
    old = os.environ.get("CESS_BLS_RLC_MSM")
    os.environ["CESS_BLS_RLC_MSM"] = "1" if request.param == "msm" else "0"
    yield request.param
    if old is None:
        os.environ.pop("CESS_BLS_RLC_MSM", None)
    else:
        os.environ["CESS_BLS_RLC_MSM"] = old


R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001


def _few_key_batch(ctx, n, nkeys, seed):
    rng = random.Random(seed)
    sks = [rng.randrange(1, R).to_bytes(32, "big") for _ in range(nkeys)]
    pks = ctx.public_keys(sks)
    owner = [rng.randrange(nkeys) for _ in range(n)]
    msgs = [rng.randbytes(32) for _ in range(n)]
    sigs = ctx.sign([sks[o] for o in owner], msgs)
    return sigs, [pks[o] for o in owner], msgs


def _pack(sigs, pks, msgs):
    offs = [0]
    for m in msgs:
        offs.append(offs[-1] + len(m))
    return b"".join(sigs), b"".join(pks), b"".join(msgs), offs


def test_rlc_all_valid_single_check(ctx):
    sigs, pks, msgs = _few_key_batch(ctx, 3000, 5, 1)
    codes, words, st = ctx.verify_rlc(*_pack(sigs, pks, msgs), seed=bytes(range(32)))
    assert set(codes) == {0}
    assert st["checks"] == 1 and st["leaves"] == 0 and st["distinct_keys"] == 5
    assert words[:3000 // 64] == [(1 << 64) - 1] * (3000 // 64)


def _fixed_len_cases(vectors):
    return [c for c in vectors["cases"] if len(bytes.fromhex(c["sig"])) == 48 and len(bytes.fromhex(c["pk"])) == 96]


def test_rlc_codes_equal_per_signature_path(ctx, vectors):
    """Forgeries, bad encodings and the golden adversarial cases spread over a
    9,000-record batch: bisection must isolate them with exact codes.  The
    expected codes come from the CONSTRUCTION (signed by the library's sign
    kernel, pinned by the reference's sign KAT: 0; forged: 5; golden record:
    its fixture code, src/lib.rs:243-246), not from another run of the
    product; the per-signature path must agree as a second check."""
    from oracle import bls_oracle
    sigs, pks, msgs = _few_key_batch(ctx, 9000, 7, 2)
    rng = random.Random(3)
    idx = rng.sample(range(9000), 12)
    want = [0] * 9000
    # forged: valid signature over another message
    msgs[idx[0]] = rng.randbytes(32)
    msgs[idx[1]] = msgs[idx[1]][:31] + bytes([msgs[idx[1]][31] ^ 1])
    # signature of another record (valid point, wrong pairing)
    sigs[idx[2]] = sigs[idx[3]]
    want[idx[0]] = want[idx[1]] = want[idx[2]] = 5
    # malformed signature encodings: the compression flag clear is no
    # compressed point (G1Affine::from_compressed fails, src/lib.rs:144 ->
    # SIG_POINT); the identity is a valid encoding whose pairing check fails
    sigs[idx[4]] = bytes([sigs[idx[4]][0] & 0x7F]) + sigs[idx[4]][1:]          # compression bit clear
    sigs[idx[5]] = b"\xc0" + bytes(47)                                         # identity signature
    with pytest.raises(bls_oracle.Invalid):
        bls_oracle.g1_from_compressed(sigs[idx[4]])
    want[idx[4]], want[idx[5]] = 2, 5
    # golden adversarial records (non-subgroup sig, off-curve key, x >= p, ...)
    cases = _fixed_len_cases(vectors)
    for j, c in zip(idx[6:], cases[:6]):
        sigs[j], msgs[j], pks[j] = bytes.fromhex(c["sig"]), bytes.fromhex(c["msg"]), bytes.fromhex(c["pk"])
        want[j] = c["code"]
    assert sorted({c["code"] for c in cases[:6]}) == [0, 2, 4, 5]
    S, P, M, offs = _pack(sigs, pks, msgs)
    codes, words, st = ctx.verify_rlc(S, P, M, offs, seed=bytes(32))
    assert list(codes) == want
    assert words[:9000 // 64] == [sum(1 << b for b in range(64) if want[64 * w + b] == 0) for w in range(9000 // 64)]
    expect, ewords = ctx.verify_fixed(S, P, M, offs)
    assert codes == expect and words == ewords
    assert st["checks"] > 1 and st["leaves"] >= 1


def test_rlc_cross_shard_combine(ctx):
    """Two shards (two contexts, as two ranks would hold): the product of the
    shards' Gt partials decides; only the failing shard bisects."""
    from cess_amd import bls
    sigs, pks, msgs = _few_key_batch(ctx, 6000, 4, 4)
    msgs[4500] = bytes(32)          # one forgery, in shard 1
    halves = [(0, 3000), (3000, 6000)]
    ctxs = [ctx, bls.Context(max_batch=1 << 14)]
    try:
        gts = []
        for c, (a, b) in zip(ctxs, halves):
            gts.append(c.rlc_begin(*_pack(sigs[a:b], pks[a:b], msgs[a:b]), seed=bytes([a & 255]) * 32))
        one = bytes(47) + b"\x01" + bytes(576 - 48)
        assert gts[0] == one and gts[1] != one
        ok = ctxs[0].gt_product_is_one(b"".join(gts))
        assert not ok
        assert ctxs[0].gt_product_is_one(gts[0] + gts[0])
        res = [c.rlc_finish(ok) for c in ctxs]
    finally:
        ctxs[1].close()
    assert set(res[0][0]) == {0} and res[0][2]["leaves"] == 0
    c1 = res[1][0]
    assert c1[1500] == 5 and c1.count(0) == 2999 and res[1][2]["leaves"] >= 1


def test_rlc_empty_and_tiny(ctx):
    codes, words, st = ctx.verify_rlc(b"", b"", b"", [0], seed=bytes(32))
    assert codes == b"" and st["checks"] == 0
    sigs, pks, msgs = _few_key_batch(ctx, 3, 1, 5)
    msgs[1] = bytes(32)
    codes, words, st = ctx.verify_rlc(*_pack(sigs, pks, msgs), seed=bytes(32))
    assert list(codes) == [0, 5, 0]


def test_rlc_bucket_sums_equal_scalar_multiples(ctx, vectors, rlc_sums_path):
    """The Gt value of one failing combination (forgery, malformed and identity
    records in it) is bit-identical whether the sums come from the buckets or
    from per-record multiples, with several key groups and 20,000 records."""
    if rlc_sums_path != "msm":
        pytest.skip("compares both paths itself")
    sigs, pks, msgs = _few_key_batch(ctx, 20000, 6, 7)
    want = [0] * 20000
    msgs[777] = bytes(32)                                        # forgery
    sigs[1234] = b"\xc0" + bytes(47)                             # identity signature
    sigs[4321] = bytes([sigs[4321][0] & 0x7F]) + sigs[4321][1:]  # malformed (compression flag clear)
    want[777], want[1234], want[4321] = 5, 5, 2
    cases = _fixed_len_cases(vectors)
    for j, c in zip(range(5000, 20000, 2500), cases):
        sigs[j], msgs[j], pks[j] = bytes.fromhex(c["sig"]), bytes.fromhex(c["msg"]), bytes.fromhex(c["pk"])
        want[j] = c["code"]
    packed = _pack(sigs, pks, msgs)
    seed = bytes(range(100, 132))
    gts, codes, stats = {}, {}, {}
    for mode in ("1", "0"):
        os.environ["CESS_BLS_RLC_MSM"] = mode
        gts[mode] = ctx.rlc_begin(*packed, seed=seed)
        codes[mode], _, stats[mode] = ctx.rlc_finish(False)
    one = bytes(47) + b"\x01" + bytes(576 - 48)
    assert gts["1"] == gts["0"] != one
    # every bisection check decides the same way on both paths (a wrong
    # sub-range sum would fail a check the other path passes)
    assert stats["1"] == stats["0"] and stats["1"]["checks"] > 1
    # codes by construction (fixture codes for the golden records), then the
    # per-signature path as a second check
    assert list(codes["1"]) == list(codes["0"]) == want
    expect, _ = ctx.verify_fixed(*packed)
    assert codes["1"] == expect


def test_rlc_bucket_path_large_batch(ctx, rlc_sums_path):
    """Default selection (env unset) on a batch large enough for the buckets
    and for the threaded key grouping (>= 2 slices of 65,536): all valid ->
    one check (a wrong group id would fail it), all codes 0; one forgery ->
    exactly that record fails."""
    if rlc_sums_path != "msm":
        pytest.skip("one run suffices")
    del os.environ["CESS_BLS_RLC_MSM"]
    sigs, pks, msgs = _few_key_batch(ctx, 140000, 4, 8)
    codes, words, st = ctx.verify_rlc(*_pack(sigs, pks, msgs), seed=bytes(32))
    assert set(codes) == {0} and st["checks"] == 1 and st["distinct_keys"] == 4
    msgs[123456] = bytes(32)
    codes, words, st = ctx.verify_rlc(*_pack(sigs, pks, msgs), seed=bytes(32))
    assert codes[123456] == 5 and codes.count(0) == 139999
    # one forgery: one failing range per level, so one leaf (16 + 5 checks below the first)
    assert st["leaves"] == 1 and st["checks"] == 1 + 16 + 5, st


def _msm_ok(covered, segs):
    """host_rlc.cpp msm_ok() under the default selection (env unset)."""
    return 0 < segs <= 256 and covered >= 64 * segs


def test_rlc_points_kept_scalar_multiple_fallback(ctx, rlc_sums_path):
    """Default selection with 141 segments for 9,000 records (< 64 records per
    segment): the batch's points are NOT kept (the first check already fails
    msm_ok) and every check takes the per-chunk multiples; codes stay exact."""
    if rlc_sums_path != "msm":
        pytest.skip("one run suffices")
    del os.environ["CESS_BLS_RLC_MSM"]
    assert not _msm_ok(9000, 140 + 1)
    sigs, pks, msgs = _few_key_batch(ctx, 9000, 140, 9)
    msgs[10] = bytes(32)
    msgs[8000] = bytes(32)
    packed = _pack(sigs, pks, msgs)
    codes, words, st = ctx.verify_rlc(*packed, seed=bytes(32))
    want = [0] * 9000
    want[10] = want[8000] = 5
    assert list(codes) == want
    expect, _ = ctx.verify_fixed(*packed)
    assert codes == expect
    assert st["distinct_keys"] == 140 and st["checks"] > 1


def test_rlc_kept_points_scale_all_at_bisection(ctx, rlc_sums_path):
    """the first check takes the buckets (so the batch's points are
    kept on the device, batch-wide Xs/Xh arrays of stride n with R.d_code /
    R.d_inf), but the first bisection level fails msm_ok, so rlc_scale_all
    computes the per-record multiples from those kept arrays.  200 key groups
    over 12,864 records: 12,864 >= 64 x 201 for the first check; the level
    splits the batch into ceil(12,864 / 2,048) = 7 ranges (host_rlc.cpp
    kRlcLeaf, kRlcFan), which meet the 200 groups in >= 200 + 6 terms, 213+
    segments, which would need >= 13,632 covered records; its ranges are
    leaves (<= 2,048 records), so the batch takes exactly 1 + 7 checks.
    Codes by construction, the per-signature path and the never-kept path
    (CESS_BLS_RLC_MSM=0) agree."""
    if rlc_sums_path != "msm":
        pytest.skip("compares both paths itself")
    n, k = 12864, 200
    fan = -(-n // 2048)
    assert fan == 7 and _msm_ok(n, k + 1) and not _msm_ok(n, fan + k + fan - 1) and 8 * k <= n
    sigs, pks, msgs = _few_key_batch(ctx, n, k, 13)
    want = [0] * n
    for j in (17, 4444, 12863):
        msgs[j] = bytes(32)
        want[j] = 5
    sigs[2000] = b"\xc0" + bytes(47)
    want[2000] = 5
    packed = _pack(sigs, pks, msgs)
    del os.environ["CESS_BLS_RLC_MSM"]
    codes, words, st = ctx.verify_rlc(*packed, seed=bytes(range(7, 39)))
    assert st["distinct_keys"] == k and st["checks"] == 1 + fan and st["leaves"] >= 1
    assert list(codes) == want
    expect, _ = ctx.verify_fixed(*packed)
    assert codes == expect
    os.environ["CESS_BLS_RLC_MSM"] = "0"
    codes0, _, st0 = ctx.verify_rlc(*packed, seed=bytes(range(7, 39)))
    assert codes0 == codes and st0 == st


def test_rlc_repeated_records(ctx, rlc_sums_path):
    """One record repeated 12,000 times among 8,000 others: a bucket then
    adds the same point to itself (the complete formulas' doubling case) and
    the check must still pass; a forged copy of it must still be isolated."""
    sigs, pks, msgs = _few_key_batch(ctx, 8000, 3, 12)
    sigs += [sigs[5]] * 12000
    pks += [pks[5]] * 12000
    msgs += [msgs[5]] * 12000
    codes, words, st = ctx.verify_rlc(*_pack(sigs, pks, msgs), seed=bytes(range(32)))
    assert set(codes) == {0} and st["checks"] == 1
    msgs[15000] = bytes(32)
    codes, words, st = ctx.verify_rlc(*_pack(sigs, pks, msgs), seed=bytes(range(32)))
    assert codes[15000] == 5 and codes.count(0) == 19999
