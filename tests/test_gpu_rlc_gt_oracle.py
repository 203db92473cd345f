"""GPU: the RLC checks' Gt value, byte for byte, against the oracle.

`cess_bls_rlc_begin` returns the 576-byte Gt value of a shard's first check
(`include/cess_bls.h`).  This file recomputes that value in the CPU oracle
(`oracle/bls_oracle.py`: the crate's hash_to_g1, G2Prepared, multi_miller_loop
and final_exponentiation, `/root/reference/utils/verify-bls-signatures/src/
lib.rs:25-31, :88-99`) from the documented scalar derivations and compares
bytes -- the GPU Gt against oracle Gt, not against another GPU path:

* key-grouped mode: r_i = SHA-256(seed32 || i as 8 big-endian bytes)[0:16]
  read as four big-endian 32-bit words k[0..3], r_i = sum k[w] 2^(32 w) with
  k[0] |= 1 (`k_rlc.hip rlc_scalar`, `include/cess_bls.h` RLC block), and the
  check  e(sum r_i sig_i, -G2) * prod_keys e(sum_{i in key} r_i H(m_i), pk);
* distinct-key mode (`CESS_BLS_F_RLC_DISTINCT`): the same digest words, a =
  k[0] | 1, b = k[1], r_i = a + b lambda with lambda = -x^2 mod r
  (`curve.hpp g1_mul_glv32`), and the check e(sum r_i sig_i, -G2) *
  prod_i e(r_i H(m_i), pk_i).
A context without a communicator uses record indices from 0 (`host_rlc.cpp
rlc_begin`).  Cases: all records valid (the Gt one), one forgery (a Gt value
that is not one: exact bytes), and two shards on two contexts, whose partials'
product (multiplied in the oracle) equals the oracle's check over both shards.
"""
import hashlib
import os
import random

import pytest

from test_gpu_rlc import R, _pack

pytestmark = pytest.mark.gpu

ONE = bytes(47) + b"\x01" + bytes(576 - 48)


def _o():
    import oracle.bls_oracle as o
    return o


def _digest_words(seed, i):
    d = hashlib.sha256(seed + i.to_bytes(8, "big")).digest()
    return [int.from_bytes(d[4 * w:4 * w + 4], "big") for w in range(4)]


def r_grouped(seed, i):
    k = _digest_words(seed, i)
    k[0] |= 1
    return sum(k[w] << (32 * w) for w in range(4))


def r_distinct(seed, i):
    o = _o()
    k = _digest_words(seed, i)
    lam = (-(o.BLS_X ** 2)) % o.R
    return ((k[0] | 1) + k[1] * lam) % o.R


def oracle_check(records, scalars):
    """Gt of e(sum r_i sig_i, -G2) * prod_pk e(sum_{i: pk} r_i H(m_i), pk) as the
    oracle's f12 value (grouping by key does not change the Gt value)."""
    o = _o()
    S, T, keys = None, {}, {}
    for (sig, pk, msg), r in zip(records, scalars):
        S = o.ec_add(o.FP, S, o.ec_mul(o.FP, o.g1_from_compressed(sig), r))
        T[pk] = o.ec_add(o.FP, T.get(pk), o.ec_mul(o.FP, o.hash_to_g1(msg), r))
        keys[pk] = o.g2_from_compressed(pk)
    terms = [(S, o._neg_g2_prepared())] + [(T[pk], o.g2_prepare(keys[pk])) for pk in T]
    return o.final_exponentiation(o.multi_miller_loop(terms))


def gt_from_bytes(b):
    o = _o()
    v = [int.from_bytes(b[48 * j:48 * j + 48], "big") for j in range(12)]
    f6 = lambda w: ((w[0], w[1]), (w[2], w[3]), (w[4], w[5]))   # noqa: E731
    return (f6(v[:6]), f6(v[6:]))


def _batch(ctx, n, nkeys, seed):
    rng = random.Random(seed)
    sks = [rng.randrange(1, R).to_bytes(32, "big") for _ in range(nkeys)]
    pks = ctx.public_keys(sks)
    owner = [j % nkeys for j in range(n)]
    msgs = [rng.randbytes(32) for _ in range(n)]
    return ctx.sign([sks[j] for j in owner], msgs), [pks[j] for j in owner], msgs


@pytest.fixture(scope="module")
def dctx():
    from cess_amd import bls
    c = bls.Context(max_batch=1 << 12, rlc_distinct=True)
    yield c
    c.close()


@pytest.fixture(params=["msm", "scale"])
def sums_path(request):
    old = os.environ.get("CESS_BLS_RLC_MSM")
    os.environ["CESS_BLS_RLC_MSM"] = "1" if request.param == "msm" else "0"
    yield request.param
    if old is None:
        os.environ.pop("CESS_BLS_RLC_MSM", None)
    else:
        os.environ["CESS_BLS_RLC_MSM"] = old


def _modes(ctx, dctx):
    # (context, scalar derivation, batch size, distinct keys)
    return {"grouped": (ctx, r_grouped, 16, 2), "distinct": (dctx, r_distinct, 9, 9)}


@pytest.mark.parametrize("mode", ["grouped", "distinct"])
def test_rlc_gt_equals_oracle(ctx, dctx, mode, sums_path):
    """All valid: the oracle's check value is one and the GPU returns its
    bytes; one forgery: the GPU's bytes equal the oracle's non-one value."""
    if mode == "distinct" and sums_path == "scale":
        pytest.skip("the distinct-key mode has one sum path")
    o = _o()
    c, rfun, n, nkeys = _modes(ctx, dctx)[mode]
    sigs, pks, msgs = _batch(ctx, n, nkeys, 40 + nkeys)
    seed = hashlib.sha256(b"gt-oracle-" + mode.encode()).digest()
    scal = [rfun(seed, i) for i in range(n)]
    gt = c.rlc_begin(*_pack(sigs, pks, msgs), seed=seed)
    c.rlc_finish(True)
    want = oracle_check(list(zip(sigs, pks, msgs)), scal)
    assert want == o.F12_ONE and o.gt_to_bytes(want) == ONE
    assert gt == ONE
    msgs[5] = b"forged message, same key and signature"
    gt = c.rlc_begin(*_pack(sigs, pks, msgs), seed=seed)
    codes, _, _ = c.rlc_finish(False)
    want = o.gt_to_bytes(oracle_check(list(zip(sigs, pks, msgs)), scal))
    assert want != ONE
    assert gt == want
    assert list(codes) == [5 if i == 5 else 0 for i in range(n)]


@pytest.mark.parametrize("mode", ["grouped", "distinct"])
def test_rlc_two_shard_partials_compose(ctx, dctx, mode):
    """Two shards on two contexts (as two ranks hold them, each numbering its
    records from 0): each partial equals the oracle's check over its shard,
    and their product equals the oracle's combined check."""
    from cess_amd import bls
    o = _o()
    c0, rfun, n, nkeys = _modes(ctx, dctx)[mode]
    sigs, pks, msgs = _batch(ctx, 2 * n, nkeys, 60 + nkeys)
    msgs[n + 3] = b"forgery in shard 1"
    c1 = bls.Context(max_batch=1 << 12, rlc_distinct=(mode == "distinct"))
    try:
        seeds = [bytes([0x5a + s]) * 32 for s in range(2)]
        parts, recs, scal = [], [], []
        for s, c in enumerate((c0, c1)):
            sl = slice(s * n, (s + 1) * n)
            parts.append(c.rlc_begin(*_pack(sigs[sl], pks[sl], msgs[sl]), seed=seeds[s]))
            recs.append(list(zip(sigs[sl], pks[sl], msgs[sl])))
            scal.append([rfun(seeds[s], i) for i in range(n)])
        assert parts[0] == ONE and parts[1] != ONE
        assert parts[1] == o.gt_to_bytes(oracle_check(recs[1], scal[1]))
        prod = o.f12_mul(gt_from_bytes(parts[0]), gt_from_bytes(parts[1]))
        assert prod == oracle_check(recs[0] + recs[1], scal[0] + scal[1])
        assert not c0.gt_product_is_one(parts[0] + parts[1])
        for c in (c0, c1):
            c.rlc_finish(False)
    finally:
        c1.close()
