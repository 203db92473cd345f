"""Benchmark: verified BLS12-381 signatures/s on MI355X (BASELINE.json metric).

Workload (N=1): BASELINE config[1] — 1,048,576 independent signatures with
distinct random keys over 32-byte messages, per-signature two-pairing verify,
inputs resident in HBM.  N>1 (torch.distributed.run, one process per GPU):
weak scaling, each rank verifies its own 1M-signature shard, then the verdict
bitmap words are all-gathered over RCCL (xGMI) so every rank holds the full
batch bitmap (BASELINE config[2] shape).

A "step" = one verify_batch over the whole shard + the bitmap all-gather.
Keys/signatures are generated on the GPU with the library's own keygen/sign
kernels (untimed); a sample is checked against the CPU oracle in the tests.

Prints ONE JSON line on rank 0 (contract in the task brief), including
`roofline` (dominant kernel vs the v_mad_u64_u32 peak) and `cpu_baseline`
(the oracle timed on the host cores on a bounded sample).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# v_mad_u64_u32 peak (integer-multiply roofline): 256 CUs x 64 lanes/clk (half
# rate; measured 53 lane-ops/CU/clk at the nominal clock by tools/mad_peak.hip,
# profiles/r01_mad_peak.txt) x 2.4 GHz.
PEAK_MADS = 256 * 64 * 2.4e9
ALG_MADS_PER_FP_MUL = 288   # 12^2 (a*b) + 12^2 (m*p) 32x32-bit limb products


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--n", type=int, default=1 << 20, help="signatures per GPU")
    ap.add_argument("--forged-frac", type=float, default=0.0)
    ap.add_argument("--cpu-sample", type=int, default=384, help="records for the CPU oracle baseline (0: skip)")
    ap.add_argument("--cpu-procs", type=int, default=16)
    return ap.parse_args()


def load_opcount():
    with open(os.path.join(ROOT, "profiles", "opcount.json")) as f:
        return json.load(f)


def load_pmc_traffic():
    """HBM bytes per launch of the dominant kernel from the committed rocprofv3
    PMC summary (profiles/*_pmc_traffic.json), if one exists."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_traffic.json")))
    if not files:
        return None
    with open(files[-1]) as f:
        return json.load(f)


def make_dataset(ctx, n, seed, forged_frac):
    import numpy as np
    rng = np.random.default_rng(seed)
    sk = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    sk[:, 0] &= 0x3F          # < 2^254 < r
    sk[:, 31] |= 1            # nonzero
    msgs = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    sks = [bytes(r) for r in sk]
    pks = ctx.public_keys(sks)
    sign_msgs = msgs.copy()
    forged = np.zeros(n, dtype=bool)
    if forged_frac > 0:
        idx = rng.choice(n, size=max(1, int(n * forged_frac)), replace=False)
        forged[idx] = True
        sign_msgs[idx, 0] ^= 0xFF      # valid signature over a different message
    sigs = ctx.sign(sks, [bytes(r) for r in sign_msgs])
    return b"".join(sigs), b"".join(pks), msgs.tobytes(), forged


def _oracle_verify(rec):
    from oracle import bls_oracle as o
    return o.verify_code(*rec)


def cpu_baseline(sample, procs):
    """CPU oracle (pure-Python restatement, oracle/bls_oracle.py) on a bounded
    sample, one process per core."""
    import multiprocessing as mp
    if not sample:
        return None
    procs = max(1, min(procs, len(sample)))
    ctx = mp.get_context("fork")
    with ctx.Pool(procs) as pool:
        pool.map(_oracle_verify, sample[:procs])          # warm imports
        t = time.perf_counter()
        codes = pool.map(_oracle_verify, sample, chunksize=4)
        dt = time.perf_counter() - t
    return {"value": len(sample) / dt, "unit": "sigs/s", "cores": procs, "kind": "port",
            "sample": f"{len(sample)} records of the same workload (distinct keys, 32-byte msgs) "
                      f"through oracle/bls_oracle.py verify_code, {procs} processes, {dt:.1f}s wall",
            "codes_ok": sum(1 for c in codes if c == 0)}


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from cess_amd import bls
    from cess_amd.dist import gather_bitmap

    n = args.n
    ctx = bls.Context(device=local, max_batch=n, profile=True)
    S, P, M, forged = make_dataset(ctx, n, seed=(0x00C0FFEE, rank), forged_frac=args.forged_frac)
    d_sig = torch.frombuffer(bytearray(S), dtype=torch.uint8).to(dev)
    d_pk = torch.frombuffer(bytearray(P), dtype=torch.uint8).to(dev)
    d_msg = torch.frombuffer(bytearray(M), dtype=torch.uint8).to(dev)
    d_off = (torch.arange(n + 1, dtype=torch.int64) * 32).to(dev)
    d_codes = torch.empty(n, dtype=torch.uint8, device=dev)
    d_bitmap = torch.zeros((n + 63) // 64, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev)

    def step():
        ctx.verify_device(n, d_sig.data_ptr(), d_pk.data_ptr(), d_msg.data_ptr(), d_off.data_ptr(),
                          d_codes.data_ptr(), d_bitmap.data_ptr(), stream.cuda_stream)
        return gather_bitmap(d_bitmap, n * world, world) if world > 1 else d_bitmap

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    ctx.stage_times(reset=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        full = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    stages = ctx.stage_times(reset=True)   # HIP events on the launch stream, timed region only
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # correctness of the last step: local codes + the gathered bitmap
    codes = d_codes.cpu().numpy()
    import numpy as np
    exp_ok = ~forged
    local_ok = bool(((codes == 0) == exp_ok).all() and (codes[forged] == 5).all())
    popcount = int(sum(bin(int(w) & ((1 << 64) - 1)).count("1") for w in full.cpu().tolist()))
    ok_t = torch.tensor([1 if local_ok else 0], device=dev)
    if world > 1:
        dist.all_reduce(ok_t, op=dist.ReduceOp.MIN)

    if rank == 0:
        total = n * world * args.steps
        value = total / elapsed
        oc = load_opcount()
        per = oc["per_stage"]
        dom = max(stages, key=lambda k: stages[k])
        dom_ms = stages[dom] / args.steps                  # per launch (one launch per step, chunk = n)
        alg = (per[dom]["mul"] + per[dom]["sqr"]) * ALG_MADS_PER_FP_MUL * n
        achieved = alg / (dom_ms * 1e-3)
        pmc = load_pmc_traffic()
        traffic = None
        if pmc and pmc.get("kernel") == dom and pmc.get("n") == n:
            traffic = pmc.get("hbm_bytes_per_launch")
        cpu = None
        if world == 1 and args.cpu_sample > 0:
            import random
            rr = random.Random(5)
            idx = rr.sample(range(n), args.cpu_sample)
            sample = [(S[48 * i:48 * i + 48], M[32 * i:32 * i + 32], P[96 * i:96 * i + 96]) for i in idx]
            cpu = cpu_baseline(sample, args.cpu_procs)
        rec = {
            "metric": "verified BLS12-381 sigs/sec (node)",
            "value": value,
            "unit": "sigs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32 (381-bit Montgomery, 14x28-bit limb products via v_mad_u64_u32)",
            "data": "synthetic: random distinct keys + 32-byte messages, keys/sigs generated on GPU",
            "config": {"workload": f"BASELINE config[1]: {n} independent sigs per GPU, distinct keys, "
                                   f"per-sig 2-pairing verify" + (", RCCL allgather of verdict bitmap" if world > 1 else ""),
                       "sigs_per_gpu": n, "msg_bytes": 32, "forged_frac": args.forged_frac,
                       "parallelism": f"shard-by-index x{world}"},
            "verdicts_ok": bool(ok_t.item() == 1),
            "bitmap_popcount": popcount,
            "stage_ms_per_step": {k: v / args.steps for k, v in stages.items()},
            "roofline": {"bound": "valu-int", "kernel": dom, "achieved": achieved / 1e12, "peak": PEAK_MADS / 1e12,
                         "unit": "T mad/s (32x32-bit limb products, v_mad_u64_u32)",
                         "frac": achieved / PEAK_MADS, "traffic": traffic,
                         "alg_mads_per_sig": (per[dom]["mul"] + per[dom]["sqr"]) * ALG_MADS_PER_FP_MUL,
                         "whole_path_frac": oc["algorithmic_mads_per_sig"] * value / world / PEAK_MADS},
            "cpu_baseline": cpu,
        }
        print(json.dumps(rec), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
