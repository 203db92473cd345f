"""Quick stage-timing run: generate n signatures on the GPU, verify them, print per-stage ms."""
import random
import sys
import time

sys.path.insert(0, ".")
from cess_amd import bls  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
ctx = bls.Context(max_batch=n, profile=True)
rng = random.Random(1)
R = bls.R_ORDER
sks = [rng.randrange(1, R).to_bytes(32, "big") for _ in range(n)]
msgs = [rng.randbytes(32) for _ in range(n)]
t = time.time(); pks = ctx.public_keys(sks); print(f"keygen {n}: {time.time()-t:.2f}s", flush=True)
t = time.time(); sigs = ctx.sign(sks, msgs); print(f"sign {n}: {time.time()-t:.2f}s", flush=True)
S, P, M = b"".join(sigs), b"".join(pks), b"".join(msgs)
offs = [32 * i for i in range(n + 1)]
for rep in range(2):
    ctx.stage_times(reset=True)
    t = time.time()
    codes, words = ctx.verify_fixed(S, P, M, offs)
    dt = time.time() - t
    st = ctx.stage_times(reset=True)
    print(f"verify {n}: {dt:.3f}s  {n/dt:.0f} sigs/s  ok={codes.count(0)}  stages(ms)=" +
          ", ".join(f"{k}={v:.1f}" for k, v in st.items()), flush=True)
