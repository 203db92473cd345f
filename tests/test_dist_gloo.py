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
    for n in (1, 63, 64, 65, 1 << 20, 16 * (1 << 20) + 5):
        for world in (1, 2, 3, 8):
            prev = 0
            for r in range(world):
                a, b = shard_range(n, r, world)
                assert a == prev and (a % 64 == 0 or a == n)
                prev = b
            assert prev == n
