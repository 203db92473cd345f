"""CPU, world_size 2-3 (gloo rendezvous): the shard/merge code of the C ABI's
sharded entry points, run with several ranks on a host without a GPU.

Each rank opens the library's shared-memory communicator
(cess_bls_comm_open_shm -- the transport the sharded entry points use when the
ranks share a host, comm.hpp) with a name rank 0 broadcasts over gloo, stands
in the golden verdict codes of its shard (cess_bls_shard_range) and merges with
cess_bls_comm_gather_verdicts -- the same gather_verdicts() that
cess_bls_verify_batch_sharded runs after its local verification.  The merged
codes and bitmap must equal the single-process verdicts bit-exactly on every
rank, including ragged batches (a short or empty last shard).

Also: the status agreement (one failing rank fails every rank, no hang), a
batch-size mismatch across ranks (INVALID_ARG on all ranks, no hang), and a
peer that never arrives (bounded wait, CESS_BLS_E_COMM).
"""
import json
import os
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from cess_amd import bls

HERE = os.path.dirname(os.path.abspath(__file__))


def _golden_codes(n):
    """n verdict codes cycled from the oracle-generated golden fixture."""
    with open(os.path.join(HERE, "golden", "vectors.json")) as f:
        cases = json.load(f)["cases"]
    pool = [c["code"] for c in cases]
    return bytes(pool[(7 * i + i // 5) % len(pool)] for i in range(n))


def _words(codes):
    n = len(codes)
    w = [0] * ((n + 63) // 64)
    for i, c in enumerate(codes):
        if c == 0:
            w[i >> 6] |= 1 << (i & 63)
    return w


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    obj = [bls.comm_shm_name() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    return obj[0]


def _merge_worker(rank, world, port, cases, q):
    name = _init(rank, world, port)
    comm = bls.Comm(name, world, rank)
    out = []
    for n in cases:
        codes = _golden_codes(n)
        b, e, _ = bls.shard_range(n, world, rank)
        out.append(comm.gather_verdicts(n, codes[b:e]))
    # status agreement: rank world-1 fails with -3 (E_HIP), the others succeed
    agreed = comm.agree(-3 if rank == world - 1 else 0)
    all_ok = comm.agree(0)
    comm.close()
    q.put((rank, out, agreed, all_ok))
    dist.destroy_process_group()


def _run(target, world, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port) + args + (q,)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        item = q.get(timeout=120)
        res[item[0]] = item[1:]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


# ragged sizes: short last shards, an empty last shard (world 3, n = 130 ->
# 3 words over 3 ranks; n = 64 -> rank 1, 2 empty), one record, empty batch
CASES = [1000, 4096 + 5, 130, 64, 1, 0, 70000]


@pytest.mark.parametrize("world", [2, 3])
def test_gather_verdicts_matches_single(world):
    res = _run(_merge_worker, world, CASES)
    for r in range(world):
        out, agreed, all_ok = res[r]
        for n, (codes, words) in zip(CASES, out):
            exp = _golden_codes(n)
            assert codes == exp, (r, n)
            assert words == _words(exp), (r, n)
        assert agreed == -3          # one rank failed: every rank sees the failure
        assert all_ok == 0


def _mismatch_worker(rank, world, port, q):
    name = _init(rank, world, port)
    comm = bls.Comm(name, world, rank)
    n = 1000 + rank              # a caller bug: ranks disagree on the batch size
    b, e, _ = bls.shard_range(n, world, rank)
    try:
        comm.gather_verdicts(n, bytes(e - b))
        st = 0
    except bls.BlsInfraError as ex:
        st = ex.status
    # the communicator is still usable afterwards (the sequence stayed aligned)
    codes, _ = comm.gather_verdicts(128, bytes(64))
    comm.close()
    q.put((rank, st, codes == bytes(128)))
    dist.destroy_process_group()


def test_batch_size_mismatch_fails_everywhere_without_hang():
    res = _run(_mismatch_worker, 2)
    for r in range(2):
        st, after_ok = res[r]
        assert st == bls.E_INVALID_ARG
        assert after_ok


def _absent_peer_worker(name, q):
    os.environ["CESS_BLS_COMM_TIMEOUT_MS"] = "1500"
    try:
        bls.Comm(name, 2, 0)        # rank 1 never comes
        q.put(0)
    except bls.BlsInfraError as ex:
        q.put(ex.status)


def test_absent_peer_times_out():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_absent_peer_worker, args=(bls.comm_shm_name(), q))
    p.start()
    st = q.get(timeout=60)
    p.join(timeout=30)
    assert st == bls.E_COMM


def test_shard_ranges_cover_and_align():
    """cess_bls_shard_range: contiguous, word-aligned shards of equal word
    count; bench.py's config[2] shards (2 M per GPU) are exact."""
    for n in (0, 1, 63, 64, 65, 4096, 1 << 20, 16 * (1 << 20) + 5):
        for world in (1, 2, 3, 4, 8):
            wpr = ((n + 63) // 64 + world - 1) // world
            prev = 0
            for r in range(world):
                a, b, w = bls.shard_range(n, world, r)
                assert w == wpr and a == prev and (a % 64 == 0 or a == n)
                prev = b
            assert prev == n
    for world in (2, 4, 8):
        for r in range(world):
            assert bls.shard_range(world << 21, world, r)[:2] == (r << 21, (r + 1) << 21)
