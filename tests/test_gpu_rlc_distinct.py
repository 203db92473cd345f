"""GPU: distinct-key RLC (CESS_BLS_F_RLC_DISTINCT, host_rlc.cpp rlcd_*): one
Miller value per record, one final exponentiation per check, bisection over
the stored Miller values.  Parity bar as tests/test_gpu_rlc.py: the codes equal
those of the construction and of the per-signature path (src/lib.rs:243-246),
and the check's Gt value depends on the batch and seed alone (not on how
the batch is cut into launches)."""
import random

import pytest

from test_gpu_rlc import R, _fixed_len_cases, _pack

pytestmark = pytest.mark.gpu


def _distinct_batch(ctx, n, seed):
    rng = random.Random(seed)
    sks = [rng.randrange(1, R).to_bytes(32, "big") for _ in range(n)]
    pks = ctx.public_keys(sks)
    msgs = [rng.randbytes(32) for _ in range(n)]
    return ctx.sign(sks, msgs), pks, msgs


@pytest.fixture(scope="module")
def dctx():
    """A distinct-key RLC context with small launches (4,096 records), so a
    batch runs as several chunks."""
    from cess_amd import bls
    c = bls.Context(max_batch=1 << 12, rlc_distinct=True)
    yield c
    c.close()


def test_rlcd_all_valid_single_check(ctx, dctx):
    sigs, pks, msgs = _distinct_batch(ctx, 9000, 11)
    codes, words, st = dctx.verify_rlc(*_pack(sigs, pks, msgs), seed=bytes(range(32)))
    assert set(codes) == {0}
    assert st["checks"] == 1 and st["leaves"] == 0 and st["leaf_sigs"] == 0
    assert words[:9000 // 64] == [(1 << 64) - 1] * (9000 // 64)


def test_rlcd_codes_equal_per_signature_path(ctx, dctx, vectors):
    """Forgeries, malformed encodings, an identity signature and the golden
    adversarial records over 9,000 distinct-key records (three launch chunks):
    codes by construction, and equal to the per-signature path's."""
    sigs, pks, msgs = _distinct_batch(ctx, 9000, 12)
    rng = random.Random(13)
    idx = rng.sample(range(9000), 12)
    want = [0] * 9000
    msgs[idx[0]] = rng.randbytes(32)                                     # forged: another message
    sigs[idx[1]] = sigs[idx[2]]                                          # another record's signature
    want[idx[0]] = want[idx[1]] = 5
    sigs[idx[3]] = bytes([sigs[idx[3]][0] & 0x7F]) + sigs[idx[3]][1:]    # compression bit clear
    sigs[idx[4]] = b"\xc0" + bytes(47)                                   # identity signature
    want[idx[3]], want[idx[4]] = 2, 5
    cases = _fixed_len_cases(vectors)
    for j, c in zip(idx[5:], cases[:7]):
        sigs[j], msgs[j], pks[j] = bytes.fromhex(c["sig"]), bytes.fromhex(c["msg"]), bytes.fromhex(c["pk"])
        want[j] = c["code"]
    S, P, M, offs = _pack(sigs, pks, msgs)
    codes, words, st = dctx.verify_rlc(S, P, M, offs, seed=bytes(32))
    assert list(codes) == want
    expect, ewords = ctx.verify_fixed(S, P, M, offs)
    assert codes == expect and words == ewords
    assert st["checks"] > 1 and st["leaves"] >= 1


def test_rlcd_gt_independent_of_launch_chunking(ctx, dctx):
    """The check's Gt value e(sum r_i sig_i, -G2) prod_i e(r_i H_i, pk_i) is a
    property of the batch and the seed alone: the same with 4,096-record
    launches (three chunks, the S sum overlapped with the last chunk) as with
    one launch, and not one for a batch with a forgery.  (The mode's scalars
    r = a + b*lambda take 2^63 values -- soundness 2^-63 per check, as
    include/cess_bls.h states -- so its Gt differs from the key-grouped mode's,
    whose scalars are 128-bit.)"""
    from cess_amd import bls
    sigs, pks, msgs = _distinct_batch(ctx, 9000, 16)
    msgs[700] = bytes(32)
    packed = _pack(sigs, pks, msgs)
    seed = bytes([7]) * 32
    g_chunked = dctx.rlc_begin(*packed, seed=seed)
    dctx.rlc_finish(False)
    one_launch = bls.Context(max_batch=1 << 14, rlc_distinct=True)
    try:
        g_one = one_launch.rlc_begin(*packed, seed=seed)
        one_launch.rlc_finish(False)
        g_other_seed = one_launch.rlc_begin(*packed, seed=bytes([8]) * 32)
        one_launch.rlc_finish(False)
    finally:
        one_launch.close()
    one = bytes(47) + b"\x01" + bytes(576 - 48)
    assert g_chunked != one and g_chunked == g_one and g_other_seed != g_one


def test_rlcd_cross_shard_combine(ctx, dctx):
    from cess_amd import bls
    sigs, pks, msgs = _distinct_batch(ctx, 6000, 14)
    msgs[4500] = bytes(32)
    other = bls.Context(max_batch=1 << 12, rlc_distinct=True)
    try:
        gts = [dctx.rlc_begin(*_pack(sigs[:3000], pks[:3000], msgs[:3000]), seed=bytes([1]) * 32),
               other.rlc_begin(*_pack(sigs[3000:], pks[3000:], msgs[3000:]), seed=bytes([2]) * 32)]
        one = bytes(47) + b"\x01" + bytes(576 - 48)
        assert gts[0] == one and gts[1] != one
        ok = dctx.gt_product_is_one(b"".join(gts))
        assert not ok
        res = [dctx.rlc_finish(ok), other.rlc_finish(ok)]
    finally:
        other.close()
    assert set(res[0][0]) == {0} and res[0][2]["leaves"] == 0
    assert res[1][0][1500] == 5 and res[1][0].count(0) == 2999


def test_rlcd_empty_and_tiny(dctx, ctx):
    codes, words, st = dctx.verify_rlc(b"", b"", b"", [0], seed=bytes(32))
    assert codes == b"" and st["checks"] == 0
    sigs, pks, msgs = _distinct_batch(ctx, 3, 15)
    msgs[1] = bytes(32)
    codes, words, st = dctx.verify_rlc(*_pack(sigs, pks, msgs), seed=bytes(32))
    assert list(codes) == [0, 5, 0]


def test_rlc_group_fe_equals_lane_fe(ctx, dctx, monkeypatch):
    """The RLC checks' final exponentiation runs one WAVE per value (k_group_fe,
    the lane-group program); env CESS_BLS_RLC_FE=lane selects the one-lane
    k_final.  Both give the same Gt bytes, on the distinct-key check and on the
    key-grouped check, for a failing and a passing batch."""
    from cess_amd import bls
    sigs, pks, msgs = _distinct_batch(ctx, 3000, 17)
    good = _pack(sigs, pks, msgs)
    msgs[123] = bytes(32)
    bad = _pack(sigs, pks, msgs)
    grouped = bls.Context(max_batch=1 << 12)
    owner = [i % 4 for i in range(800)]
    gs = [sigs[o] for o in owner]   # placeholder signatures, replaced below
    try:
        rng = random.Random(18)
        sks = [rng.randrange(1, R).to_bytes(32, "big") for _ in range(4)]
        kp = ctx.public_keys(sks)
        gm = [rng.randbytes(32) for _ in range(800)]
        gs = ctx.sign([sks[o] for o in owner], gm)
        gm[5] = bytes(32)
        gbad = _pack(gs, [kp[o] for o in owner], gm)
        out = {}
        for fe in ("group", "lane"):
            if fe == "lane":
                monkeypatch.setenv("CESS_BLS_RLC_FE", "lane")
            res = []
            for c, packed in ((dctx, bad), (dctx, good), (grouped, gbad)):
                res.append(c.rlc_begin(*packed, seed=bytes([3]) * 32))
                c.rlc_finish(False)
            out[fe] = res
    finally:
        grouped.close()
    one = bytes(47) + b"\x01" + bytes(576 - 48)
    assert out["group"] == out["lane"]
    assert out["group"][0] != one and out["group"][1] == one and out["group"][2] != one


def test_rlcd_ragged_lanes_and_cuts(ctx, dctx):
    """4,099 records (a 4,096-record launch, then 3): the last Miller lane holds
    three records, and the bisection's cuts fall at multiples of four records
    (k_miller_rr's lanes) inside a range of 4,099.  Forgeries at a lane's
    second record, at the first record of a cut and in the ragged last lane get
    code 5; every other record 0, as the per-signature path says."""
    sigs, pks, msgs = _distinct_batch(ctx, 4099, 19)
    bad = [1365, 2732, 4098]
    for j in bad:
        msgs[j] = bytes(32)
    packed = _pack(sigs, pks, msgs)
    codes, words, st = dctx.verify_rlc(*packed, seed=bytes([5]) * 32)
    want = [5 if i in bad else 0 for i in range(4099)]
    assert list(codes) == want
    expect, ewords = ctx.verify_fixed(*packed)
    assert codes == expect and words == ewords
    assert st["checks"] > 1 and st["leaves"] >= 1
