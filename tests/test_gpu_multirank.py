"""GPU: the product's sharded entry points with TWO ranks (BASELINE config[2]'s
shard/gather path, config[3]'s Gt-partial exchange), before any 8-GPU node runs
them.

Two processes (tests/multirank_worker.py) on GPU 0 form a 2-rank communicator
over the library's host shared-memory transport (cess_bls_comm_init_shm; RCCL
refuses two ranks on one device) and run
  * cess_bls_verify_batch_sharded on ragged batches (1,000 and 4,096 + 5
    records: the last shard is short) with forgeries and the adversarial golden
    records (non-subgroup, off-curve, x >= p, bad flags, identities) in rank 1's
    shard only;
  * cess_bls_verify_batch_sharded_device on the 4,101-record batch, each rank's
    shard resident in HBM;
  * cess_bls_verify_batch_rlc_sharded with a different shard per rank and two
    forgeries on rank 1;
  * a failure on one rank only (corrupt offsets; a missing device buffer):
    every rank must return the failure (no hang), and the next call works.
  * cess_bls_verify_batch_var_sharded with the wrong-length golden records
    (SIG_LEN / PK_LEN) in rank 1's shard.
Expected codes come from the CONSTRUCTION, not from the product: a record
signed by the library's sign kernel (pinned by the reference's sign KAT) is 0,
a forgery 5, an injected golden record its fixture code (every fixed-length
golden case: non-subgroup, off-curve, x >= p, bad flags, the (O, O) identity
pairs, precedence).  The gathered codes and bitmaps must equal them on both
ranks, and a single-context run must equal them too.  Reference axis: one
verdict per (sig, msg, key) as verify_bls_signature
(utils/verify-bls-signatures/src/lib.rs:243-246).
"""
import json
import os
import random
import subprocess
import sys

import numpy as np
import pytest

from cess_amd import bls

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
WORLD = 2


def _signed(ctx, n, seed, keys=None):
    rng = random.Random(seed)
    if keys is None:
        sks = [rng.randrange(1, R).to_bytes(32, "big") for _ in range(n)]
    else:
        ks = [rng.randrange(1, R).to_bytes(32, "big") for _ in range(keys)]
        sks = [ks[rng.randrange(keys)] for _ in range(n)]
    msgs = [rng.randbytes(32) for _ in range(n)]
    return ctx.sign(sks, msgs), msgs, ctx.public_keys(sks)


def _offs(msgs):
    o = [0]
    for m in msgs:
        o.append(o[-1] + len(m))
    return np.asarray(o, dtype=np.uint64)


def _rank1_adversarial(vectors, sigs, msgs, pks, lo, seed):
    """Every fixed-length golden record plus 10 forgeries at indices >= lo
    (rank 1's shard); returns the records and their codes by construction."""
    rng = random.Random(seed)
    cases = [c for c in vectors["cases"] if len(c["sig"]) == 96 and len(c["pk"]) == 192]
    assert any(c["name"].startswith("identity_pair") for c in cases)      # (O, O) records among them
    idx = rng.sample(range(lo, len(sigs)), len(cases) + 10)
    expect = [0] * len(sigs)
    for c, i in zip(cases, idx):
        sigs[i], msgs[i], pks[i] = bytes.fromhex(c["sig"]), bytes.fromhex(c["msg"]), bytes.fromhex(c["pk"])
        expect[i] = c["code"]
    for i in idx[len(cases):]:
        msgs[i] = bytes(b ^ 0x5A for b in msgs[i])      # forgeries
        expect[i] = 5
    return sigs, msgs, pks, bytes(expect)


def _words(codes):
    n = len(codes)
    return [sum(1 << b for b in range(64) if 64 * w + b < n and codes[64 * w + b] == 0) for w in range((n + 63) // 64)]


def _arr(b):
    return np.frombuffer(b, dtype=np.uint8)


@pytest.fixture(scope="module")
def multirank(ctx, vectors, tmp_path_factory):
    tmp = tmp_path_factory.mktemp("multirank")
    data, expect = {}, {}
    for case, n in (("a", 1000), ("b", 4096 + 5)):
        lo = bls.shard_range(n, WORLD, 1)[0]
        sigs, msgs, pks, want = _rank1_adversarial(vectors, *_signed(ctx, n, 40 + n), lo=lo, seed=n)
        S, P, M, o = b"".join(sigs), b"".join(pks), b"".join(msgs), _offs(msgs)
        codes, words = ctx.verify_fixed(S, P, M, o)
        assert codes == want and words == _words(want)       # single context vs construction
        assert set(want[:lo]) == {0} and set(want[lo:]) == {0, 2, 4, 5}   # the bad records are all in rank 1's shard
        data.update({f"{case}_S": _arr(S), f"{case}_P": _arr(P), f"{case}_M": _arr(M), f"{case}_o": o,
                     f"{case}_n": np.uint64(n)})
        expect[case] = (want, _words(want))
        if case == "a":
            # the var-length batch: case a's records with the wrong-length golden
            # records inserted into rank 1's shard
            recs = list(zip(sigs, msgs, pks))
            vw = list(want)
            for j, c in enumerate(vectors["length_cases"]):
                at = len(recs) - 3 - 37 * j
                recs.insert(at, (bytes.fromhex(c["sig"]), bytes.fromhex(c["msg"]), bytes.fromhex(c["pk"])))
                vw.insert(at, c["code"])
            assert bls.shard_range(len(recs), WORLD, 1)[0] < len(recs) - 3 - 37 * 6
            for k, part in enumerate(zip(*recs)):
                data[f"var_{k}"] = _arr(b"".join(part))
                data[f"var_{k}_o"] = _offs(part)
            expect["var"] = (bytes(vw), _words(vw))
    for r, n in ((0, 1500), (1, 1700)):
        sigs, msgs, pks = _signed(ctx, n, 60 + r, keys=3)
        if r == 1:
            msgs[17] = bytes(32)
            msgs[1600] = bytes(31) + b"\x01"
        S, P, M, o = b"".join(sigs), b"".join(pks), b"".join(msgs), _offs(msgs)
        data.update({f"rlc{r}_S": _arr(S), f"rlc{r}_P": _arr(P), f"rlc{r}_M": _arr(M), f"rlc{r}_o": o})
        want = bytes(5 if (r == 1 and i in (17, 1600)) else 0 for i in range(n))
        assert ctx.verify_fixed(S, P, M, o) == (want, _words(want))
        expect[f"rlc{r}"] = (want, _words(want))
    path = str(tmp / "data.npz")
    np.savez(path, **data)
    name = bls.comm_shm_name()
    env = dict(os.environ, CESS_BLS_COMM_TIMEOUT_MS="60000", HSA_ENABLE_IPC_MODE_LEGACY="0")
    procs = [subprocess.Popen([sys.executable, "-u", os.path.join(HERE, "multirank_worker.py"), "--rank", str(r),
                               "--world", str(WORLD), "--name", name, "--data", path,
                               "--out", str(tmp / f"rank{r}.json")], env=env)
             for r in range(WORLD)]
    codes = []
    for p in procs:
        try:
            codes.append(p.wait(timeout=240))
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    assert codes == [0] * WORLD, codes
    out = []
    for r in range(WORLD):
        with open(tmp / f"rank{r}.json") as f:
            out.append(json.load(f))
    return out, expect


def test_transport_is_shm(multirank):
    out, _ = multirank
    assert [o["kind"] for o in out] == ["shm"] * WORLD


@pytest.mark.parametrize("case", ["a", "b"])
def test_host_sharded_equals_construction(multirank, case):
    out, expect = multirank
    codes, words = expect[case]
    for o in out:
        assert bytes.fromhex(o[f"host_{case}"]["codes"]) == codes
        assert o[f"host_{case}"]["words"] == words


def test_var_sharded_wrong_lengths(multirank):
    out, expect = multirank
    codes, words = expect["var"]
    assert {1, 3} <= set(codes)
    for o in out:
        assert bytes.fromhex(o["var"]["codes"]) == codes
        assert o["var"]["words"] == words


def test_device_sharded_equals_construction(multirank):
    out, expect = multirank
    codes, words = expect["b"]
    for o in out:
        assert bytes.fromhex(o["device_b"]["codes"]) == codes
        assert o["device_b"]["words"] == words
        assert all(w == 0 for w in o["device_b"]["pad_words"])   # the short last shard's unused words


def test_one_rank_failure_fails_every_rank(multirank):
    out, expect = multirank
    for o in out:
        assert o["host_bad_offsets_status"] == bls.E_INVALID_ARG
        assert o["device_bad_status"] == bls.E_INVALID_ARG
        assert bytes.fromhex(o["host_after_failure"]["codes"]) == expect["a"][0]


def test_rlc_sharded_two_ranks(multirank):
    out, expect = multirank
    for r, o in enumerate(out):
        codes, words = expect[f"rlc{r}"]
        assert bytes.fromhex(o["rlc"]["codes"]) == codes
        assert o["rlc"]["words"] == words
        assert o["rlc"]["stats"]["global_ok"] is False          # rank 1's forgeries fail the combined product
    assert out[0]["rlc"]["stats"]["leaf_sigs"] == 0            # rank 0's own check passed: no bisection
    assert out[1]["rlc"]["stats"]["leaf_sigs"] > 0
    assert expect["rlc1"][0][17] == 5 and expect["rlc1"][0][1600] == 5


def test_control_collectives(multirank):
    out, _ = multirank
    assert [o["max"] for o in out] == [WORLD - 0.5] * WORLD
