"""GPU parity of the keyed batch (distinct-key table, include/cess_bls.h
cess_bls_keys_load / cess_bls_verify_batch_keyed): per-key decode
(src/lib.rs:68-82) and G2Prepared (:88) done once per distinct key must give
the same per-signature codes as verify_bls_signature (:243-247) on the
expanded records — golden fixtures included (bad keys, identity keys, the
signature-first precedence)."""
import random

import pytest

pytestmark = pytest.mark.gpu


def _fixed_cases(vectors):
    return [c for c in vectors["cases"] if len(c["sig"]) == 96 and len(c["pk"]) == 192]


def _keyed(ctx, recs):
    keys = sorted({r[2] for r in recs})
    kid = {k: j for j, k in enumerate(keys)}
    kc = ctx.load_keys(keys)
    msgs = [r[1] for r in recs]
    offs = [0]
    for m in msgs:
        offs.append(offs[-1] + len(m))
    codes, words = ctx.verify_keyed(b"".join(r[0] for r in recs), [kid[r[2]] for r in recs], b"".join(msgs), offs)
    return kc, keys, codes, words


def test_keyed_golden_codes(ctx, vectors):
    cases = _fixed_cases(vectors)
    recs = [(bytes.fromhex(c["sig"]), bytes.fromhex(c["msg"]), bytes.fromhex(c["pk"])) for c in cases]
    kc, keys, codes, words = _keyed(ctx, recs)
    assert list(codes) == [c["code"] for c in cases]
    for i, c in enumerate(codes):
        assert (words[i // 64] >> (i % 64)) & 1 == (c == 0)
    assert set(kc) <= {0, 4}


def test_keyed_few_keys_matches_per_signature(ctx):
    """Audit-round shape (BASELINE config[3]: few keys) with forgeries, through
    a chunked context: keyed codes == per-record codes."""
    from cess_amd import bls
    rng = random.Random(7)
    R = bls.R_ORDER
    sks = [rng.randrange(1, R).to_bytes(32, "big") for _ in range(5)]
    pks = ctx.public_keys(sks)
    n = 700
    who = [rng.randrange(5) for _ in range(n)]
    msgs = [bytes(rng.randrange(256) for _ in range(32)) for _ in range(n)]
    sign_msgs = list(msgs)
    for i in (3, 64, 65, 699):
        sign_msgs[i] = bytes(32)
    sigs = ctx.sign([sks[w] for w in who], sign_msgs)
    small = bls.Context(max_batch=128)
    try:
        kc = small.load_keys(pks)
        assert kc == bytes(5)
        codes, words = small.verify_keyed(b"".join(sigs), who, b"".join(msgs), [32 * i for i in range(n + 1)])
    finally:
        small.close()
    ref, ref_words = ctx.verify_fixed(b"".join(sigs), b"".join(pks[w] for w in who), b"".join(msgs),
                                      [32 * i for i in range(n + 1)])
    assert codes == ref and words == ref_words
    assert [i for i, c in enumerate(codes) if c] == [3, 64, 65, 699]


def test_keyed_rejects_bad_index(ctx):
    from cess_amd import bls
    ctx.load_keys([bytes.fromhex("c0") + bytes(95)])
    with pytest.raises(bls.BlsInfraError):
        ctx.verify_keyed(bytes(48), [1], b"", [0, 0])


def test_verify_batch_dedups_keys(ctx, vectors):
    """The Python mirror's verify_batch routes few-key batches through the key
    table; verdicts equal the per-record path, golden bad keys included."""
    from cess_amd import bls
    cases = _fixed_cases(vectors)
    recs = [(bytes.fromhex(c["sig"]), bytes.fromhex(c["msg"]), bytes.fromhex(c["pk"])) for c in cases]
    recs = (recs * (1 + 2048 // max(len(recs), 1)))[:2048]
    assert 8 * len({r[2] for r in recs}) <= len(recs)
    c = bls.Context(max_batch=4096)      # no caller-loaded key table: the dedup path runs
    try:
        v = bls.verify_batch(recs, ctx=c)
        assert c._keys_owner == "verify_batch"
    finally:
        c.close()
    ref = bls.verify_batch(recs, ctx=ctx, dedup_keys=False)
    assert v.codes == ref.codes and v.bitmap == ref.bitmap
