"""GPU: the multi-GPU and boundary surface of the C ABI.

* RCCL communicator owned by the library: a 1-rank communicator
  (cess_bls_comm_id / _comm_init) drives the sharded entry points (host and
  device-resident) and the RLC Gt-partial all-gather; verdicts equal the
  single-context path.  (N > 1 ranks run in bench.py on the driver's 8-GPU
  node; the launcher and shard layout are CPU-tested in test_launcher.py.)
* A multi-device context over devices [0, 0] (two sub-contexts on one GPU)
  shards host batches across host threads: codes equal the single context.
* Config: strict identity (KeyValidate) flag; cp_enclave_verify::verify_bls
  wrapper (key first, distinct statuses where the reference panics).
* Advisor findings: RLC bisects on a local failure whatever the combined
  verdict; many distinct keys; out-of-range device key indices; verify_batch
  never overwrites a caller's key table.
"""
import random

import numpy as np
import pytest

from cess_amd import bls

pytestmark = pytest.mark.gpu

R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001


def _signed(ctx, n, seed, keys=None, msg_len=32):
    rng = random.Random(seed)
    if keys is None:
        sks = [rng.randrange(1, R).to_bytes(32, "big") for _ in range(n)]
    else:
        ks = [rng.randrange(1, R).to_bytes(32, "big") for _ in range(keys)]
        sks = [ks[rng.randrange(keys)] for _ in range(n)]
    msgs = [rng.randbytes(msg_len) for _ in range(n)]
    return ctx.sign(sks, msgs), msgs, ctx.public_keys(sks)


def _offs(msgs):
    o = [0]
    for m in msgs:
        o.append(o[-1] + len(m))
    return o


def _with_adversarial(vectors, sigs, msgs, pks, seed, k=40):
    rng = random.Random(seed)
    cases = [c for c in vectors["cases"] if len(c["sig"]) == 96 and len(c["pk"]) == 192]
    n = len(sigs)
    for j, i in enumerate(rng.sample(range(n), k)):
        c = cases[j % len(cases)]
        sigs[i], msgs[i], pks[i] = bytes.fromhex(c["sig"]), bytes.fromhex(c["msg"]), bytes.fromhex(c["pk"])
    for i in rng.sample(range(n), 5):
        msgs[i] = rng.randbytes(len(msgs[i]) or 1)   # forgeries (or already-bad records)
    return sigs, msgs, pks


@pytest.fixture(scope="module")
def comm_ctx():
    c = bls.Context(max_batch=4096)
    c.comm_init(1, 0, bls.comm_id())
    yield c
    c.close()


def test_comm_single_rank_sharded(ctx, comm_ctx, vectors):
    sigs, msgs, pks = _with_adversarial(vectors, *_signed(ctx, 700, 31), seed=32)
    S, P, M, o = b"".join(sigs), b"".join(pks), b"".join(msgs), _offs(msgs)
    expect, ewords = ctx.verify_fixed(S, P, M, o)
    assert set(expect) - {0} and 0 in expect
    codes, words = comm_ctx.verify_sharded(S, P, M, o)
    assert codes == expect and words == ewords
    # device-resident sharded form: this rank's shard is the whole batch
    n = len(sigs)
    b, e, wpr = bls.shard_range(n, 1, 0)
    assert (b, e, wpr) == (0, n, (n + 63) // 64)
    d = [comm_ctx.to_device(x) for x in (S, P, M, np.asarray(o, dtype=np.uint64))]
    dc, dw = comm_ctx.device_alloc(wpr * 64), comm_ctx.device_alloc(wpr * 8)
    try:
        comm_ctx.verify_sharded_device(n, d[0], d[1], d[2], d[3], dc, dw)
        comm_ctx.synchronize()
        assert comm_ctx.from_device(dc, n) == expect
        got = np.frombuffer(comm_ctx.from_device(dw, wpr * 8), dtype=np.uint64).tolist()
        assert got == ewords
    finally:
        for p in d + [dc, dw]:
            comm_ctx.device_free(p)
    assert comm_ctx.comm_max(3.25) == 3.25
    comm_ctx.comm_barrier()


def test_comm_rlc_sharded(ctx, comm_ctx):
    sigs, msgs, pks = _signed(ctx, 3000, 33, keys=5)
    msgs[1234] = bytes(32)                          # one forgery
    S, P, M, o = b"".join(sigs), b"".join(pks), b"".join(msgs), _offs(msgs)
    expect, _ = ctx.verify_fixed(S, P, M, o)
    codes, words, st = comm_ctx.verify_rlc_sharded(S, P, M, o)
    assert codes == expect and expect[1234] == 5
    assert st["global_ok"] is False and st["leaf_sigs"] > 0
    sigs[1234] = ctx.sign([bytes(31) + b"\x07"], [msgs[1234]])[0]   # a valid signature by another key: still 5
    codes2, _, st2 = comm_ctx.verify_rlc_sharded(b"".join(sigs), P, M, o)
    assert codes2[1234] == 5


def test_multi_device_context(ctx, vectors):
    m = bls.Context(max_batch=1024, devices=[0, 0])
    try:
        sigs, msgs, pks = _with_adversarial(vectors, *_signed(ctx, 2500, 34), seed=35)
        recs = list(zip(sigs, msgs, pks)) + [(bytes.fromhex(c["sig"]), bytes.fromhex(c["msg"]),
                                              bytes.fromhex(c["pk"])) for c in vectors["length_cases"]]
        assert m.verify_codes(recs) == ctx.verify_codes(recs)
        S, P, M, o = b"".join(sigs), b"".join(pks), b"".join(msgs), _offs(msgs)
        assert m.verify_fixed(S, P, M, o) == ctx.verify_fixed(S, P, M, o)
        # RLC across the two devices equals the per-signature path
        k_sigs, k_msgs, k_pks = _signed(ctx, 2600, 36, keys=3)
        k_msgs[7] = bytes(32)
        k_msgs[2599] = bytes(32)
        KS, KP, KM, ko = b"".join(k_sigs), b"".join(k_pks), b"".join(k_msgs), _offs(k_msgs)
        codes, _, st = m.verify_rlc(KS, KP, KM, ko)
        assert codes == ctx.verify_fixed(KS, KP, KM, ko)[0]
        # generators and the keyed batch through the multi-device context
        sks = [random.Random(37 + i).randrange(1, R).to_bytes(32, "big") for i in range(300)]
        assert m.public_keys(sks) == ctx.public_keys(sks)
        keys = sorted(set(k_pks))
        m.load_keys(keys)
        idx = [keys.index(p) for p in k_pks]
        assert m.verify_keyed(KS, idx, KM, ko)[0] == ctx.verify_fixed(KS, KP, KM, ko)[0]
    finally:
        m.close()


def test_strict_identity_flag(ctx, vectors):
    ident = next(c for c in vectors["cases"] if c["sig"].startswith("c0") and c["pk"].startswith("c0"))
    O_sig, O_pk = bytes.fromhex(ident["sig"]), bytes.fromhex(ident["pk"])
    sigs, msgs, pks = _signed(ctx, 4, 38)
    recs = [(O_sig, msgs[0], O_pk), (sigs[1], msgs[1], O_pk), (sigs[2], msgs[2], pks[2]), (O_sig, msgs[3], pks[3])]
    assert list(ctx.verify_codes(recs)) == [0, 5, 0, 5]          # reference: identity keys accepted
    s = bls.Context(max_batch=256, strict_identity=True)
    try:
        assert list(s.verify_codes(recs)) == [4, 4, 0, 5]        # KeyValidate: identity key rejected
        s.load_keys([O_pk, pks[2]])
        assert s.verify_keyed(b"".join([sigs[1], sigs[2]]), [0, 1], msgs[1] + msgs[2], [0, 32, 64])[0] == bytes([4, 0])
    finally:
        s.close()


def test_enclave_verify_bls(ctx, vectors):
    sigs, msgs, pks = _signed(ctx, 2, 39)
    assert ctx.enclave_verify_bls(pks[0], msgs[0], sigs[0]) is True
    assert ctx.enclave_verify_bls(pks[0], msgs[1], sigs[0]) is False
    bad_key = next(c for c in vectors["cases"] if c["code"] == 4)
    bad_sig = next(c for c in vectors["cases"] if c["code"] == 2)
    for key, sig, st in [(bytes.fromhex(bad_key["pk"]), bytes.fromhex(bad_sig["sig"]), bls.E_BAD_KEY),
                         (pks[0][:95], sigs[0], bls.E_BAD_KEY),
                         (pks[0], bytes.fromhex(bad_sig["sig"]), bls.E_BAD_SIG),
                         (pks[0], sigs[0] + b"\x00", bls.E_BAD_SIG)]:
        with pytest.raises(bls.BlsInfraError) as ei:
            ctx.enclave_verify_bls(key, msgs[0], sig)
        assert ei.value.status == st


def test_keyed_device_out_of_range_index(ctx):
    sigs, msgs, pks = _signed(ctx, 128, 40, keys=4)
    keys = sorted(set(pks))
    c = bls.Context(max_batch=256)
    try:
        c.load_keys(keys)
        idx = np.array([keys.index(p) for p in pks], dtype=np.uint32)
        idx[5], idx[77] = 7, 0xFFFFFFFF
        S, M = b"".join(sigs), b"".join(msgs)
        d = [c.to_device(S), c.to_device(idx), c.to_device(M), c.to_device(np.asarray(_offs(msgs), dtype=np.uint64))]
        dc, dw = c.device_alloc(128), c.device_alloc(16)
        c.verify_keyed_device(128, d[0], d[1], d[2], d[3], dc, dw)
        c.synchronize()
        codes = c.from_device(dc, 128)
        for p in d + [dc, dw]:
            c.device_free(p)
    finally:
        c.close()
    assert codes[5] == 4 and codes[77] == 4
    assert all(codes[i] == 0 for i in range(128) if i not in (5, 77))


def test_rlc_local_failure_bisects_despite_global_ok(ctx):
    """A shard whose own check failed must bisect even if the caller reports
    the combined product as one (a faulty peer / corrupted all-gather)."""
    sigs, msgs, pks = _signed(ctx, 2500, 41, keys=2)
    msgs[999] = bytes(32)
    S, P, M, o = b"".join(sigs), b"".join(pks), b"".join(msgs), _offs(msgs)
    c = bls.Context(max_batch=4096)
    try:
        gt = c.rlc_begin(S, P, M, o)
        assert gt != bytes(47) + b"\x01" + bytes(528)
        codes, words, st = c.rlc_finish(True)          # caller claims global_ok = 1
    finally:
        c.close()
    assert codes[999] == 5 and codes.count(0) == 2499


@pytest.mark.parametrize("nkeys,forged", [(1000, [3, 1500, 3999]), (1024, [10, 9000])])
def test_rlc_many_keys(ctx, nkeys, forged):
    """K > n/8: per-signature fallback; K = n/16: bisection over term lists
    (no NR x K replication): 16,384 records split into 8 ranges of 2,048, of
    which at most the two holding a forgery are verified per signature."""
    n = 4000 if nkeys == 1000 else 16384
    sigs, msgs, pks = _signed(ctx, n, 42 + nkeys, keys=nkeys)
    for i in forged:
        msgs[i] = bytes(32)
    S, P, M, o = b"".join(sigs), b"".join(pks), b"".join(msgs), _offs(msgs)
    expect, _ = ctx.verify_fixed(S, P, M, o)
    codes, _, st = ctx.verify_rlc(S, P, M, o)
    assert codes == expect
    assert [i for i in range(n) if codes[i]] == sorted(forged)
    if nkeys * 8 > n:
        assert st["leaf_sigs"] == n                     # verified per signature
    else:
        assert st["leaf_sigs"] < n // 2


def test_verify_batch_keeps_user_key_table(vectors):
    c = bls.Context(max_batch=1024)
    try:
        sigs, msgs, pks = _signed(c, 600, 43, keys=3)
        user_keys = sorted(set(pks))[::-1]
        c.load_keys(user_keys)
        msgs[17] = bytes(32)
        v = bls.verify_batch(list(zip(sigs, msgs, pks)), ctx=c)     # few keys, but the table is the caller's
        assert v.codes[17] == 5 and v.codes.count(0) == 599
        idx = [user_keys.index(p) for p in pks]
        codes, _ = c.verify_keyed(b"".join(sigs), idx, b"".join(msgs), _offs(msgs))
        assert codes == v.codes
    finally:
        c.close()


def test_comm_info_single_rank(comm_ctx):
    """The communicator reports its own size and rank (ncclCommCount /
    ncclCommUserRank) and the PCI bus id of each rank's device."""
    info = comm_ctx.comm_info()
    assert info["nranks"] == 1 and info["rank"] == 0
    assert len(info["bus_ids"]) == 1 and ":" in info["bus_ids"][0]
    assert comm_ctx.comm_info(bus_ids=False) == {"nranks": 1, "rank": 0}


def test_var_sharded_single_rank(ctx, comm_ctx, vectors):
    """Arbitrary-length records through the sharded var entry point: the
    wrong-length golden records get their SIG_LEN / PK_LEN codes."""
    sigs, msgs, pks = _signed(ctx, 600, 44)
    recs = list(zip(sigs, msgs, pks))
    fx = [(bytes.fromhex(c["sig"]), bytes.fromhex(c["msg"]), bytes.fromhex(c["pk"]), c["code"])
          for c in vectors["length_cases"] + vectors["cases"]]
    for j, (s, m, k, _) in enumerate(fx):
        recs.insert(7 * j + 3, (s, m, k))
    expect = [0] * len(recs)
    for j, f in enumerate(fx):
        expect[7 * j + 3] = f[3]
    codes, words = comm_ctx.verify_var_sharded(recs)
    assert list(codes) == expect
    assert {1, 3} <= set(codes)
    assert words == [sum(1 << b for b in range(64) if w * 64 + b < len(recs) and codes[w * 64 + b] == 0)
                     for w in range((len(recs) + 63) // 64)]


LONE_RANK = r"""
import os, sys, time
sys.path.insert(0, sys.argv[1])
from cess_amd import bls
bls.load_library()
c = bls.Context(max_batch=256)
t0 = time.time()
try:
    c.comm_init(2, 0, bls.comm_id())      # rank 1 never arrives
    print("STATUS 0", time.time() - t0)
except bls.BlsInfraError as ex:
    print("STATUS", ex.status, time.time() - t0, flush=True)
c.close()
print("CLOSED", flush=True)
os._exit(0)   # RCCL's bootstrap thread stays blocked: end with _exit (include/cess_bls.h)
"""


def test_rccl_lone_rank_fails_within_deadline():
    """A rank whose peer never arrives: the non-blocking RCCL init is polled
    against CESS_BLS_COMM_TIMEOUT_MS, aborted, and returns CESS_BLS_E_COMM --
    a non-zero exit instead of a hang in the first 8-GPU run."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, CESS_BLS_COMM_TIMEOUT_MS="4000", HSA_ENABLE_IPC_MODE_LEGACY="0")
    p = subprocess.run([sys.executable, "-c", LONE_RANK, root], env=env, capture_output=True, text=True, timeout=100)
    line = [x for x in p.stdout.splitlines() if x.startswith("STATUS")]
    assert p.returncode == 0 and line and "CLOSED" in p.stdout, (p.returncode, p.stdout[-2000:], p.stderr[-2000:])
    _, st, dt = line[-1].split()
    assert int(st) == bls.E_COMM, line
    assert 3.5 < float(dt) < 60, line
