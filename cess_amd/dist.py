"""Multi-GPU sharding of a verification batch (one process per GPU) for
callers that already run a torch.distributed process group.

The product path does NOT need this module: the C-ABI library owns an RCCL
communicator (cess_bls_comm_init) and all-gathers verdict bitmaps, codes and
RLC Gt partials itself (cess_bls_verify_batch_sharded*, _rlc_sharded), which is
what bench.py and C/Rust callers use.  This module restates the same shard
layout (cess_bls_shard_range) and protocol over torch.distributed (gloo on CPU
in the tests, RCCL/"nccl" on GPUs).

Signatures are independent (reference src/lib.rs:243 is per signature), so a
batch shards by index with no exchange during compute.  The only collective is
the all-gather of the per-rank verdict-bitmap words, which gives every rank the
full batch bitmap -- what a node-side caller of verify_batch needs.
"""
from __future__ import annotations

from typing import Tuple


def shard_range(n: int, rank: int, world: int, align: int = 64) -> Tuple[int, int]:
    """Contiguous [start, end) of rank's shard, the layout of the library's
    cess_bls_shard_range: ceil(n / 64) bitmap words split into `world` equal
    runs of ceil(words / world) words (the last shards may be short or empty),
    so every shard is whole bitmap words and an all-gather of equal-size blocks
    concatenates to the batch bitmap with no re-packing."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    words = (n + align - 1) // align
    per = (words + world - 1) // world
    return min(n, rank * per * align), min(n, (rank + 1) * per * align)


def gather_bitmap(local_words, n: int, world: int, group=None):
    """All-gather per-rank bitmap words (int64 tensor on the rank's device) into
    the full batch bitmap (ceil(n/64) words).  Shards from shard_range are
    word-aligned, so concatenation in rank order is the global bitmap."""
    import torch
    import torch.distributed as dist

    if world == 1:
        return local_words
    words = (n + 63) // 64
    mx = (words + world - 1) // world
    buf = torch.zeros(mx, dtype=torch.int64, device=local_words.device)
    buf[: local_words.numel()] = local_words
    out = torch.empty(world * mx, dtype=torch.int64, device=local_words.device)
    if dist.get_backend(group) == "gloo":
        parts = [torch.empty_like(buf) for _ in range(world)]
        dist.all_gather(parts, buf, group=group)
        out = torch.cat(parts)
    else:
        dist.all_gather_into_tensor(out, buf, group=group)
    return out[:words]


def shard_seed(seed: bytes, rank: int) -> bytes:
    """Per-rank RLC seed.  The scalars r_i are derived from (seed, local index);
    without a rank-specific seed two ranks would reuse the same r_i, letting an
    adversary cancel errors across shards."""
    import hashlib
    return hashlib.sha256(b"cess-rlc-shard" + seed + rank.to_bytes(4, "little")).digest()


def verify_rlc_sharded(ctx, sigs: bytes, pks: bytes, msgs: bytes, msg_offsets, seed: bytes,
                       rank: int, world: int, device=None, group=None):
    """RLC batch mode across ranks: every rank checks its shard
    and contributes its Gt partial; the partials are all-gathered (RCCL over
    xGMI; gloo on CPU) and multiplied on the device for the batch-level
    verdict; a rank bisects iff its OWN check failed (rlc_finish), so no other
    rank's partial can cancel a local failure.  Arguments are this rank's shard
    (fixed-stride records); returns (codes, bitmap words, stats) for the shard.
    `seed` must be secret and unpredictable to the signers (include/cess_bls.h)."""
    import torch
    import torch.distributed as dist

    gt = ctx.rlc_begin(sigs, pks, msgs, msg_offsets, shard_seed(seed, rank))
    if world == 1:
        gts = gt
    else:
        dev = device if device is not None else torch.device("cpu")
        mine = torch.tensor(list(gt), dtype=torch.uint8, device=dev)
        parts = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(parts, mine, group=group)
        gts = b"".join(bytes(p.cpu().tolist()) for p in parts)
    ok = ctx.gt_product_is_one(gts)
    codes, words, stats = ctx.rlc_finish(ok)
    stats = dict(stats, global_ok=ok)
    return codes, words, stats
