"""Records whose Miller-loop value lies in a proper subfield.

With secret key 1 the key is the G2 generator and the signature is H(m), so the
two Miller loops run over (H, -G2) and (H, G2): the lines of -T are the
p^6-conjugates of the lines of T (up to Fp2 factors), f = conj(g) g lies in
Fp6 and the easy part of the final exponentiation gives m = 1 although f != 1.
Every compressed power of the hard part is then zero (z2 = z3 = 0), which
takes the final exponentiation's Granger-Scott fallback (bls/pair_fe.hpp
pcyc_chain `degen`, bls/staged.hpp cyc_chain, and k_group's program in the
lane-group shape).  Secret key r - 1 (key -G2, signature -H(m)) does the same.
These are valid signatures for the reference (src/lib.rs:243-247; the oracle
confirms m = 1 and code 0 for both keys): code 0 and the identity Gt.  The
same signature against another message is a forgery: code 5."""
import pytest

import oracle.bls_oracle as o

pytestmark = pytest.mark.gpu

MSGS = [b"", b"subfield miller value", bytes(range(32)), b"\xa5" * 100]
SKS = [1, o.R - 1]


def _records(ctx):
    sks = [k.to_bytes(32, "big") for k in SKS for _ in MSGS]
    msgs = [m for _ in SKS for m in MSGS]
    pks = ctx.public_keys(sks)
    sigs = ctx.sign(sks, msgs)
    return sks, msgs, pks, sigs


def test_subfield_keys_and_signatures(ctx):
    sks, msgs, pks, sigs = _records(ctx)
    g2 = o.g2_to_compressed(o.G2_GEN)
    ng2 = o.g2_to_compressed(o.ec_neg(o.FP2, o.G2_GEN))
    assert pks == [g2] * len(MSGS) + [ng2] * len(MSGS)
    for m, s in zip(MSGS, sigs[: len(MSGS)]):
        assert s == o.g1_to_compressed(o.hash_to_g1(m))


def test_subfield_miller_value_verifies(ctx):
    _, msgs, pks, sigs = _records(ctx)
    recs = list(zip(sigs, msgs, pks))
    one = o.gt_to_bytes(o.F12_ONE)
    codes, gts = ctx.gt(recs)
    assert list(codes) == [0] * len(recs)
    assert all(g == one for g in gts)
    assert list(ctx.verify_codes(recs)) == [0] * len(recs)


def test_subfield_signature_on_other_message_is_forgery(ctx):
    _, msgs, pks, sigs = _records(ctx)
    # each signature against the next message under the same key
    recs = [(sigs[i], msgs[(i + 1) % len(MSGS) + (i // len(MSGS)) * len(MSGS)], pks[i]) for i in range(len(sigs))]
    one = o.gt_to_bytes(o.F12_ONE)
    codes, gts = ctx.gt(recs)
    assert list(codes) == [5] * len(recs)
    assert all(g != one for g in gts)
