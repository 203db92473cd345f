"""Count Fp multiplies/squares per signature per stage, from the device source
compiled for the host (tests/hostemu/emu.cpp with -DCESS_COUNT_OPS).
Writes profiles/opcount.json (the algorithmic-work denominator of bench.py)."""
import ctypes
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
lib_path = "/tmp/libemu_count.so"
subprocess.check_call(["g++", "-O2", "-std=c++17", "-DCESS_HOSTEMU", "-DCESS_COUNT_OPS", "-shared", "-fPIC",
                       os.path.join(ROOT, "tests", "hostemu", "emu.cpp"), "-o", lib_path])
L = ctypes.CDLL(lib_path)
vec = json.load(open(os.path.join(ROOT, "tests", "golden", "vectors.json")))
stages = ["k_decode_sig", "k_decode_pk", "k_hash", "k_prepare", "k_miller", "k_final"]
rows = []
for c in vec["cases"]:
    if c["code"] != 0 or not c["name"].startswith("valid_len32"):
        continue
    out = (ctypes.c_uint64 * 12)()
    m = bytes.fromhex(c["msg"])
    L.emu_opcount(bytes.fromhex(c["sig"]), m, len(m), bytes.fromhex(c["pk"]), out)
    rows.append([(out[2 * i] / 2, out[2 * i + 1]) for i in range(6)])   # mul in half units
avg = {st: {"mul": sum(r[i][0] for r in rows) / len(rows), "sqr": sum(r[i][1] for r in rows) / len(rows)}
       for i, st in enumerate(stages)}
tot_m = sum(v["mul"] for v in avg.values())
tot_s = sum(v["sqr"] for v in avg.values())
res = {
    "what": "Fp multiplies and squarings per valid signature (32-byte message), per kernel; "
            "algorithmic unit = one 381-bit Montgomery product = 288 32x32-bit limb products (12^2 a*b + 12^2 m*p); "
            "a lazily reduced Fp2 product (3 products, 2 reductions) counts as 2.5 multiplies",
    "samples": len(rows), "per_stage": avg, "total_mul": tot_m, "total_sqr": tot_s,
    "algorithmic_mads_per_sig": (tot_m + tot_s) * 288,
    "issued_mads_per_sig": tot_m * 392 + tot_s * 301,
}
# generator side: k_sign (PrivateKey::sign) over the golden keygen/sign records
srows = []
for g in vec["keygen_sign"]:
    out = (ctypes.c_uint64 * 2)()
    m = bytes.fromhex(g["msg"])
    L.emu_opcount_sign(bytes.fromhex(g["sk"]), m, len(m), out)
    srows.append((out[0] / 2, out[1]))
res["generator"] = {"k_sign": {"mul": sum(r[0] for r in srows) / len(srows),
                               "sqr": sum(r[1] for r in srows) / len(srows), "samples": len(srows)}}
# the distinct-key RLC's Miller lane loop (k_miller_rr, four records per lane)
# over four valid golden records, per record
valid = [c for c in vec["cases"] if c["code"] == 0 and len(c["msg"]) == 64 and len(c["pk"]) == 192]
if len(valid) >= 4:
    rr = (ctypes.c_uint64 * 2)()
    L.emu_opcount_rr(b"".join(bytes.fromhex(c["msg"]) for c in valid[:4]),
                     b"".join(bytes.fromhex(c["pk"]) for c in valid[:4]), rr)
    res["rlcd"] = {"k_miller_rr": {"mul": rr[0] / 2 / 4, "sqr": rr[1] / 4, "records_per_lane": 4,
                                   "what": "per record: one general sparse product per line and a quarter of "
                                           "the lane's accumulator squarings"}}
os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
json.dump(res, open(os.path.join(ROOT, "profiles", "opcount.json"), "w"), indent=1)
print(json.dumps(res, indent=1))
