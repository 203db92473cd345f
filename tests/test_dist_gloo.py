"""CPU, world_size 2 (gloo): the sharding + bitmap all-gather used by bench.py
for N GPUs (cess_amd/dist.py).  Each rank stands in its verdict words for its
shard; the gathered bitmap must equal the single-process bitmap."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from cess_amd.dist import gather_bitmap, shard_range


def _expected_words(n, bad):
    words = [0] * ((n + 63) // 64)
    for i in range(n):
        if i not in bad:
            words[i >> 6] |= 1 << (i & 63)
    return [w - (1 << 64) if w >= (1 << 63) else w for w in words]


def _worker(rank, world, port, n, bad, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    a, b = shard_range(n, rank, world)
    words = [0] * ((b - a + 63) // 64)
    for i in range(a, b):
        if i not in bad:
            j = i - a
            words[j >> 6] |= 1 << (j & 63)
    local = torch.tensor([w - (1 << 64) if w >= (1 << 63) else w for w in words], dtype=torch.int64)
    full = gather_bitmap(local, n, world)
    q.put((rank, full.tolist()))
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("n,world", [(1000, 2), (4096, 2), (130, 2), (5000, 3)])
def test_gather_matches_single(n, world):
    bad = {0, 63, 64, n // 2, n - 1}
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, bad, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    exp = _expected_words(n, bad)
    for r in range(world):
        assert res[r] == exp


def test_shard_ranges_cover_and_align():
    for n in (0, 1, 63, 64, 65, 1 << 20, 16 * (1 << 20) + 5):
        for world in (1, 2, 3, 8):
            prev = 0
            for r in range(world):
                a, b = shard_range(n, r, world)
                assert a == prev and (a % 64 == 0 or a == n)
                prev = b
            assert prev == n


def test_shard_ranges_match_library():
    """dist.shard_range restates the C ABI's cess_bls_shard_range (a pure
    function: callable without a GPU); bench.py's config[2] shards are exact."""
    from cess_amd import bls
    for n in (0, 1, 63, 64, 65, 4096, 1 << 20, 16 * (1 << 20) + 5, 16 << 20):
        for world in (1, 2, 3, 4, 8):
            wpr = ((n + 63) // 64 + world - 1) // world
            for r in range(world):
                assert bls.shard_range(n, world, r) == shard_range(n, r, world) + (wpr,)
    for world in (2, 4, 8):   # config[2]: 2 M per GPU
        for r in range(world):
            assert bls.shard_range(world << 21, world, r)[:2] == (r << 21, (r + 1) << 21)


# --- RLC orchestration (cess_amd.dist.verify_rlc_sharded) ------------------
GT_ONE = bytes(47) + b"\x01" + bytes(528)


class _ShardCtx:
    """Stand-in for a GPU context: a record is 'valid' iff its message byte 0
    is even.  The Gt partial is one iff the shard is all valid (the algebra is
    the GPU's; this checks the cross-rank protocol).  rlc_finish follows the
    library: a shard bisects iff its own check failed, whatever the combined
    verdict (bisection then yields exact codes)."""

    def rlc_begin(self, sigs, pks, msgs, offs, seed):
        self.seed = seed
        self.valid = [msgs[offs[i]] % 2 == 0 for i in range(len(offs) - 1)]
        return GT_ONE if all(self.valid) else b"\x02" + bytes(575)

    def gt_product_is_one(self, gts):
        return all(gts[i:i + 576] == GT_ONE for i in range(0, len(gts), 576))

    def rlc_finish(self, ok):
        local_ok = all(self.valid)
        codes = bytes(0 if (local_ok or v) else 5 for v in self.valid)
        return codes, [], {"checks": 1}


def _rlc_worker(rank, world, port, n, bad, q):
    from cess_amd.dist import verify_rlc_sharded
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    a, b = shard_range(n, rank, world)
    msgs = bytes(1 if i in bad else 2 for i in range(a, b))
    ctx = _ShardCtx()
    codes, _, st = verify_rlc_sharded(ctx, b"", b"", msgs, list(range(b - a + 1)), b"s" * 32, rank, world)
    q.put((rank, codes, st["global_ok"], ctx.seed))
    dist.destroy_process_group()


@pytest.mark.parametrize("bad", [set(), {700}])
def test_rlc_sharded_protocol(bad):
    n, world = 1000, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rlc_worker, args=(r, world, port, n, bad, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, codes, ok, seed = q.get(timeout=120)
        res[r] = (codes, ok, seed)
    for p in procs:
        p.join(timeout=60)
    assert res[0][2] != res[1][2]                      # per-rank scalars
    assert all(res[r][1] == (not bad) for r in range(world))
    full = res[0][0] + res[1][0]
    assert [i for i in range(n) if full[i] != 0] == sorted(bad)
