"""One rank of tests/test_gpu_multirank.py (not a test module itself).

Runs the C ABI's sharded entry points -- cess_bls_verify_batch_sharded,
cess_bls_verify_batch_sharded_device, cess_bls_verify_batch_rlc_sharded -- as
rank `--rank` of `--world` over the host shared-memory transport
(cess_bls_comm_init_shm), all ranks on GPU 0, and writes what every call
returned to `--out` (JSON).  The batches come from `--data` (an .npz the parent
test wrote).
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rank", type=int, required=True)
    ap.add_argument("--world", type=int, required=True)
    ap.add_argument("--name", required=True)
    ap.add_argument("--data", required=True)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()

    from cess_amd import bls
    bls.load_library()
    import numpy as np

    data = np.load(a.data, allow_pickle=False)
    ctx = bls.Context(device=0, max_batch=1024)     # chunks: the shards run as several launches
    ctx.comm_init_shm(a.world, a.rank, a.name)
    out = {"rank": a.rank, "kind": ctx.comm_kind}

    def status_of(fn):
        try:
            return 0, fn()
        except bls.BlsInfraError as ex:
            return ex.status, None

    # host-buffer sharded batches: every rank passes the whole batch
    for case in ("a", "b"):
        S, P, M, o = (bytes(data[f"{case}_S"]), bytes(data[f"{case}_P"]), bytes(data[f"{case}_M"]),
                      data[f"{case}_o"])
        codes, words = ctx.verify_sharded(S, P, M, o)
        out[f"host_{case}"] = {"codes": codes.hex(), "words": [int(w) for w in words]}

    # arbitrary-length records (wrong-length golden records in rank 1's shard)
    parts = [bytes(data[f"var_{k}"]) for k in range(3)]
    offs = [data[f"var_{k}_o"] for k in range(3)]
    recs = [tuple(parts[k][int(offs[k][i]):int(offs[k][i + 1])] for k in range(3)) for i in range(len(offs[0]) - 1)]
    codes, words = ctx.verify_var_sharded(recs)
    out["var"] = {"codes": codes.hex(), "words": [int(w) for w in words]}

    # a failure on one rank (rank 1 corrupts its copy of the offsets inside its
    # shard) fails the call on EVERY rank, then the communicator still works
    S, P, M = bytes(data["a_S"]), bytes(data["a_P"]), bytes(data["a_M"])
    o = data["a_o"].copy()
    if a.rank == 1:
        o[701] = o[700] + 10 ** 6
    st, _ = status_of(lambda: ctx.verify_sharded(S, P, M, o))
    out["host_bad_offsets_status"] = st
    codes, words = ctx.verify_sharded(S, P, M, data["a_o"])
    out["host_after_failure"] = {"codes": codes.hex(), "words": [int(w) for w in words]}

    # device-resident sharded batch: this rank's shard in HBM, the gathered
    # verdicts of the whole batch in HBM
    n = int(data["b_n"])
    b, e, wpr = bls.shard_range(n, a.world, a.rank)
    Sb, Pb, Mb, ob = data["b_S"], data["b_P"], data["b_M"], data["b_o"]
    mo = ob[b:e + 1] - ob[b]
    d = [ctx.to_device(np.ascontiguousarray(x)) for x in
         (Sb[48 * b:48 * e], Pb[96 * b:96 * e], Mb[ob[b]:ob[e]], mo.astype(np.uint64))]
    dc = ctx.device_alloc(a.world * wpr * 64)
    dw = ctx.device_alloc(a.world * wpr * 8)
    ctx.verify_sharded_device(n, d[0], d[1], d[2], d[3], dc, dw)
    ctx.synchronize()
    codes_all = ctx.from_device(dc, a.world * wpr * 64)
    words_all = np.frombuffer(ctx.from_device(dw, a.world * wpr * 8), dtype=np.uint64)
    out["device_b"] = {"codes": codes_all[:n].hex(), "words": [int(w) for w in words_all[:(n + 63) // 64]],
                       "pad_words": [int(w) for w in words_all[(n + 63) // 64:]]}
    # a device-path failure on one rank (rank 1: no signature buffer) fails every rank
    st, _ = status_of(lambda: ctx.verify_sharded_device(n, 0 if a.rank == 1 else d[0], d[1], d[2], d[3], dc, dw))
    out["device_bad_status"] = st
    for p in d + [dc, dw]:
        ctx.device_free(p)

    # RLC over the communicator: each rank checks its own shard, Gt partials
    # all-gathered and multiplied, bisection iff the rank's own check failed
    R = f"rlc{a.rank}"
    codes, words, stt = ctx.verify_rlc_sharded(bytes(data[f"{R}_S"]), bytes(data[f"{R}_P"]), bytes(data[f"{R}_M"]),
                                               data[f"{R}_o"])
    out["rlc"] = {"codes": codes.hex(), "words": [int(w) for w in words],
                  "stats": {k: (bool(v) if isinstance(v, bool) else int(v)) for k, v in stt.items()}}

    out["max"] = ctx.comm_max(float(a.rank) + 0.5)
    ctx.comm_barrier()
    ctx.close()
    with open(a.out, "w") as f:
        json.dump(out, f)


if __name__ == "__main__":
    main()
