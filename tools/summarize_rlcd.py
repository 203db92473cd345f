"""Summarise a tools/profile_rlcd.sh run (gpurun_out/prof_<tag>_rlcd) into
profiles/<tag>_rlcd_rocprof_kernel_stats.csv and <tag>_rlcd_pmc_traffic.json:
HBM bytes per full-size launch of each profiled kernel (the launches with the
largest grid: one chunk of records), bytes = (2 FETCH_SIZE + WRITE_SIZE) KiB
(gfx950 correction, as tools/summarize_prof.py).  bench.py --mode rlcd reads
the JSON whose lib_sha256 equals the benched library's.
Usage: python tools/summarize_rlcd.py <tag>"""
import csv
import glob
import json
import os
import shutil
import sys

tag = sys.argv[1]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = os.path.join(root, "gpurun_out", f"prof_{tag}_rlcd")
dst = os.path.join(root, "profiles")
stats = glob.glob(os.path.join(src, "trace", "**", "*kernel_stats.csv"), recursive=True)
if stats:
    shutil.copy(stats[0], os.path.join(dst, f"{tag}_rlcd_rocprof_kernel_stats.csv"))
rows = {}
for f in glob.glob(os.path.join(src, "pmc_*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        key = (k, r["Counter_Name"], r["Dispatch_Id"])
        rows.setdefault(key, [int(r["Grid_Size"]), 0.0])
        rows[key][1] += float(r["Counter_Value"])
out = {"source": f"profiles/{tag}_rlcd_pmc_traffic.json", "mode": "rlcd",
       "lib_sha256": open(os.path.join(src, "lib_sha256.txt")).read().split()[0], "all": {}}
for k in sorted({k for k, _, _ in rows}):
    grid = max(g for (kk, _, _), (g, _) in rows.items() if kk == k)
    d = {"grid": grid}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        v = [val for (kk, cc, _), (g, val) in rows.items() if kk == k and cc == c and g == grid]
        if v:
            d[c] = sum(v) / len(v)
    if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
        d["hbm_bytes_per_launch"] = (2 * d["FETCH_SIZE"] + d["WRITE_SIZE"]) * 1024
    out["all"][k] = d
json.dump(out, open(os.path.join(dst, f"{tag}_rlcd_pmc_traffic.json"), "w"), indent=1)
print(json.dumps(out, indent=1))
