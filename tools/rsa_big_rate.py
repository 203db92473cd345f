"""Throughput of the loop-form RSA class (2049-4096-bit moduli, k_rsa_verify_big)
on one MI355X: the fixture's valid signatures under the 3072- and 4096-bit keys
(tests/golden/rsa_vectors.json) replicated to a batch, device-resident records,
codes checked against the fixture.  Usage (GPU box): python tools/rsa_big_rate.py [records]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from cess_amd import bls  # noqa: E402

rv = json.load(open(os.path.join(ROOT, "tests", "golden", "rsa_vectors.json")))
N = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 16
ctx = bls.Context(max_batch=N)
for bits in (2048, 3072, 4096):
    ki = next(i for i, k in enumerate(rv["keys"]) if k["bits"] == bits and k["e"] == 65537)
    pool = [c for c in rv["cases"] if c["key"] == ki and c["code"] == 0]
    n = N
    recs = [pool[i % len(pool)] for i in range(n)]
    S = b"".join(bytes.fromhex(r["sig"]) for r in recs)
    M = b"".join(bytes.fromhex(r["msg"]) for r in recs)
    so = np.cumsum([0] + [len(r["sig"]) // 2 for r in recs]).astype(np.uint64)
    mo = np.cumsum([0] + [len(r["msg"]) // 2 for r in recs]).astype(np.uint64)
    assert ctx.rsa_keys_load([bytes.fromhex(rv["keys"][ki]["spki"])] + [bytes.fromhex(rv["keys"][2]["spki"])] * 5000) \
        [0] == 0   # many keys in the table: the unsorted lists (the big class never takes the key-uniform path)
    d = [ctx.to_device(np.zeros(n, dtype=np.uint32)), ctx.to_device(S), ctx.to_device(so), ctx.to_device(M),
         ctx.to_device(mo)]
    dc = ctx.device_alloc(n)
    ctx.rsa_verify_batch_device(n, *d, dc)
    ctx.synchronize()
    t0 = time.perf_counter()
    reps = 3
    for _ in range(reps):
        ctx.rsa_verify_batch_device(n, *d, dc)
    ctx.synchronize()
    dt = (time.perf_counter() - t0) / reps
    ok = ctx.from_device(dc, n) == bytes(n)
    print(json.dumps({"bits": bits, "records": n, "sigs_per_s": n / dt, "ms": dt * 1e3, "codes_ok": ok}))
    for p in d + [dc]:
        ctx.device_free(p)
ctx.close()
