"""Single-call and small-batch latency of the verifier through the C ABI on
cuda:0, with the lane-group small-batch path (k_group, one signature per wave)
and without it (CESS_BLS_SMALL_BATCH=0: the one-lane-per-signature pipeline
for every batch).  Also the decode-only deserialize calls.  Prints one line
per measurement: median / p90 wall time per call (host buffers incl. PCIe)
and the resulting sigs/s; the last line is a JSON summary."""
import ctypes
import json
import os
import random
import statistics
import sys
import time

sys.path.insert(0, ".")
from cess_amd import bls  # noqa: E402

SIZES = [int(x) for x in os.environ.get("LAT_SIZES", "1,8,64,256,1024,2048,4096,8192,16384").split(",")]
n = max(SIZES)
gen = bls.Context(max_batch=65536)
rng = random.Random(3)
sks = [rng.randrange(1, bls.R_ORDER).to_bytes(32, "big") for _ in range(n)]
msgs = [rng.randbytes(32) for _ in range(n)]
pks = gen.public_keys(sks)
sigs = gen.sign(sks, msgs)
msgs[5] = bytes(32)                       # one forgery in every batch of >= 8
gen.close()
lib = bls.load_library()
summary = {}


def timed(fn, reps):
    fn()
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t)
    ts.sort()
    return statistics.median(ts), ts[int(0.9 * (len(ts) - 1))]


for mode, small in (("group", None), ("pipeline", "0")):
    if small is None:
        os.environ.pop("CESS_BLS_SMALL_BATCH", None)
    else:
        os.environ["CESS_BLS_SMALL_BATCH"] = small
    ctx = bls.Context(max_batch=65536, profile=True)
    code = (ctypes.c_uint8 * 1)()
    buf = lambda b: (ctypes.c_uint8 * len(b)).from_buffer_copy(b)  # noqa: E731
    s0, m0, p0 = buf(sigs[0]), buf(msgs[0]), buf(pks[0])

    def one():
        rc = lib.cess_bls_verify(ctx._h, s0, 48, m0, 32, p0, 96, code)
        assert rc == 0 and code[0] == 0
    med, p90 = timed(one, 50)
    ctx.stage_stats(reset=True)
    one()
    st = {k: round(v[0], 3) for k, v in ctx.stage_stats(reset=True).items() if v[1]}
    print(f"[{mode}] cess_bls_verify (1 sig): median {med * 1e3:.2f} ms  p90 {p90 * 1e3:.2f} ms "
          f"-> {1 / med:.0f} sigs/s  stages(ms) {st}", flush=True)
    summary[f"{mode}_verify1_ms"] = med * 1e3
    summary[f"{mode}_verify1_stages_ms"] = st
    for b in SIZES:
        recs = list(zip(sigs[:b], msgs[:b], pks[:b]))
        want = bytes(5 if (i == 5) else 0 for i in range(b))
        med, p90 = timed(lambda: (lambda c: c == want or (_ for _ in ()).throw(AssertionError("codes")))(
            ctx.verify_codes(recs)), 5 if b <= 4096 else 3)
        print(f"[{mode}] batch {b}: median {med * 1e3:.2f} ms  p90 {p90 * 1e3:.2f} ms -> {b / med:.0f} sigs/s",
              flush=True)
        summary[f"{mode}_batch{b}_ms"] = med * 1e3
    if mode == "group":
        for kind, enc in ((bls.KIND_SIG, sigs[0]), (bls.KIND_PK, pks[0])):
            med, p90 = timed(lambda: ctx.deserialize_codes(kind, [enc]), 20)
            nm = "sig" if kind == bls.KIND_SIG else "pk"
            print(f"[{mode}] deserialize 1 {nm}: median {med * 1e3:.2f} ms p90 {p90 * 1e3:.2f} ms", flush=True)
            summary[f"deserialize1_{nm}_ms"] = med * 1e3
    ctx.close()
print(json.dumps(summary))
