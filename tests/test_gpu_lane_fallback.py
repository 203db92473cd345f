"""GPU parity of the one-lane fallback kernels (k_miller / k_final, selected with
CESS_BLS_MILLER=lane / CESS_BLS_FINAL=lane; the defaults are the lane-pair
k_miller2 / k_final2).  The choice is read once per process (host.cpp
miller_pair / final_pair), so each case runs in a child process on the
pipeline path (CESS_BLS_SMALL_BATCH=0) and checks the golden codes and Gt
bytes of tests/golden/vectors.json, and the subfield records of
tests/test_gpu_subfield.py (the degenerate decompression) -- the fallbacks
share the final exponentiation program (bls/staged.hpp, CESS_CHAIN_TAIL) with
the host emulation of the CPU tests."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, sys
sys.path.insert(0, sys.argv[1])
from cess_amd import bls
vec = json.load(open(sys.argv[2]))
ctx = bls.Context(max_batch=1 << 12)
cases = vec["cases"]
recs = [(bytes.fromhex(c["sig"]), bytes.fromhex(c["msg"]), bytes.fromhex(c["pk"])) for c in cases]
codes = ctx.verify_codes(recs)
bad = [(c["name"], c["code"], int(codes[i])) for i, c in enumerate(cases) if codes[i] != c["code"]]
gcases = [c for c in cases if "gt" in c]
grecs = [(bytes.fromhex(c["sig"]), bytes.fromhex(c["msg"]), bytes.fromhex(c["pk"])) for c in gcases]
gcodes, gts = ctx.gt(grecs)
gbad = [c["name"] for i, c in enumerate(gcases) if gcodes[i] != c["code"] or gts[i].hex() != c["gt"]]
# secret keys 1 and r - 1: Miller value in Fp6, m = 1, the degenerate chain
# (tests/test_gpu_subfield.py); valid, Gt = 1
one = gcases and [gts[i] for i, c in enumerate(gcases) if c["code"] == 0][0]
R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
sks = [k.to_bytes(32, "big") for k in (1, R - 1) for _ in range(2)]
msgs = [b"", b"subfield miller value"] * 2
srecs = list(zip(ctx.sign(sks, msgs), msgs, ctx.public_keys(sks)))
scodes, sgts = ctx.gt(srecs)
sbad = [i for i in range(len(srecs)) if scodes[i] != 0 or sgts[i] != one]
ctx.close()
print(json.dumps({"n": len(cases), "bad": bad, "ngt": len(gcases), "gbad": gbad, "sbad": sbad}))
"""


@pytest.mark.parametrize("miller,final", [("lane", "lane"), ("lane", "pair"), ("pair", "lane")])
def test_lane_fallback_golden(miller, final):
    env = dict(os.environ, CESS_BLS_SMALL_BATCH="0")
    for k, v in (("CESS_BLS_MILLER", miller), ("CESS_BLS_FINAL", final)):
        if v == "lane":
            env[k] = "lane"
        else:
            env.pop(k, None)
    out = subprocess.run([sys.executable, "-c", CHILD, ROOT, os.path.join(ROOT, "tests", "golden", "vectors.json")],
                         env=env, capture_output=True, text=True, timeout=180)
    assert out.returncode == 0, out.stderr[-2000:]
    r = json.loads(out.stdout.strip().splitlines()[-1])
    assert r["n"] > 50 and r["ngt"] >= 8, r
    assert not r["bad"], r["bad"]
    assert not r["gbad"], r["gbad"]
    assert not r["sbad"], r["sbad"]
