"""Single-call and small-batch latency of the verifier through the C ABI on
cuda:0 (VERDICT r01 'boundary looseness': cess_bls_verify runs the whole
six-kernel pipeline for one signature).  Prints one line per batch size:
median / p90 wall time per call and the resulting sigs/s."""
import ctypes
import random
import statistics
import sys
import time

sys.path.insert(0, ".")
from cess_amd import bls  # noqa: E402

ctx = bls.Context(max_batch=65536)
rng = random.Random(3)
n = 65536
sks = [rng.randrange(1, bls.R_ORDER).to_bytes(32, "big") for _ in range(n)]
msgs = [rng.randbytes(32) for _ in range(n)]
pks = ctx.public_keys(sks)
sigs = ctx.sign(sks, msgs)
lib = bls.load_library()
code = (ctypes.c_uint8 * 1)()
buf = lambda b: (ctypes.c_uint8 * len(b)).from_buffer_copy(b)
S1 = [buf(x) for x in sigs[:200]]
M1 = [buf(x) for x in msgs[:200]]
P1 = [buf(x) for x in pks[:200]]
for _ in range(20):   # warm-up of the single-call path
    lib.cess_bls_verify(ctx._h, S1[0], 48, M1[0], 32, P1[0], 96, code)
times = []
for i in range(200):
    t = time.perf_counter()
    rc = lib.cess_bls_verify(ctx._h, S1[i], 48, M1[i], 32, P1[i], 96, code)
    times.append(time.perf_counter() - t)
    assert rc == 0 and code[0] == 0
med, p90 = statistics.median(times), sorted(times)[int(0.9 * len(times))]
print(f"cess_bls_verify (1 sig): median {med * 1e3:.2f} ms  p90 {p90 * 1e3:.2f} ms  -> {1 / med:.0f} sigs/s", flush=True)
for b in (64, 1024, 16384, 65536):
    recs = list(zip(sigs[:b], msgs[:b], pks[:b]))
    ctx.verify_codes(recs)
    ts = []
    for _ in range(5):
        t = time.perf_counter()
        c = ctx.verify_codes(recs)
        ts.append(time.perf_counter() - t)
        assert bytes(c) == bytes(b)
    m = statistics.median(ts)
    print(f"verify_codes batch {b}: median {m * 1e3:.2f} ms per call (host buffers incl. PCIe) -> {b / m:.0f} sigs/s",
          flush=True)
ctx.close()
