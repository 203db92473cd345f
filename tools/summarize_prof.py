"""Summarise a tools/profile.sh run (gpurun_out/prof_<tag>) into profiles/:
  <tag>_rocprof_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary
  <tag>_pmc_summary.txt            per-kernel PMC values (one launch each)
  <tag>_pmc_traffic.json           HBM bytes per launch (gfx950 correction:
                                   FETCH_SIZE reports 1/2 of wide reads, so
                                   bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024)
Usage: python tools/summarize_prof.py <tag> [n]"""
import csv
import glob
import json
import os
import shutil
import sys

tag = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = os.path.join(root, "gpurun_out", f"prof_{tag}")
dst = os.path.join(root, "profiles")
stats = glob.glob(os.path.join(src, "trace", "**", "*kernel_stats.csv"), recursive=True)
if stats:
    shutil.copy(stats[0], os.path.join(dst, f"{tag}_rocprof_kernel_stats.csv"))
# Per-dispatch attribution: a kernel's counters come from its dispatches over
# the whole batch (grid = n) only -- e.g. the 64-thread k_prepare dispatch that
# builds the -G2 table at context creation is excluded.  Counter values of one
# dispatch are summed over its rows (XCD / SE instances).
agg = {}
for f in glob.glob(os.path.join(src, "pmc_*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        # (grid = n, or n plus the padding of a wave-padded list: k_rsa_verify_2048u;
        # the lane-pair kernels k_miller2 / k_final2 run two lanes per record: 2n)
        g = int(r["Grid_Size"])
        if not (n <= g <= n + (1 << 18) or 2 * n <= g <= 2 * n + 256):
            continue
        k = r["Kernel_Name"].split("(")[0]
        d = agg.setdefault(k, {"grid": int(r["Grid_Size"]), "vgpr": int(r["VGPR_Count"]),
                               "agpr": int(r.get("Accum_VGPR_Count", 0) or 0),
                               "scratch_per_lane": int(r["Scratch_Size"]), "lds": int(r["LDS_Block_Size"]),
                               "_dispatches": {}})
        cnt = d["_dispatches"].setdefault(r["Counter_Name"], set())
        cnt.add(r["Dispatch_Id"])
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
for d in agg.values():   # per launch: divide by the number of full-batch dispatches of that counter's pass
    for c, ids in d.pop("_dispatches").items():
        d[c] /= len(ids)
sha_file = os.path.join(src, "lib_sha256.txt")
lib_sha = open(sha_file).read().split()[0] if os.path.exists(sha_file) else None
out = {"n": n, "source": f"profiles/{tag}_pmc_summary.txt", "lib_sha256": lib_sha, "all": {}}
lines = [f"# rocprofv3 PMC summary, tag {tag} (bench.py --n {n} --steps 1 --warmup 0; per full-batch launch; "
         f"libcess_bls.so sha256 {lib_sha})",
         "# separate passes: FETCH_SIZE | WRITE_SIZE | SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE",
         "# HBM bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024  (FETCH_SIZE in KiB; gfx950 FETCH_SIZE reports 1/2 of wide reads)"]
for k, d in sorted(agg.items()):
    hbm = None
    if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
        hbm = (2 * d["FETCH_SIZE"] + d["WRITE_SIZE"]) * 1024
    out["all"][k] = {"hbm_bytes_per_launch": hbm, **{c: v for c, v in d.items()}}
    extra = ""
    if "SQ_INSTS_VALU" in d and "SQ_WAVES" in d:
        extra = f" SQ_INSTS_VALU/wave={d['SQ_INSTS_VALU'] / d['SQ_WAVES']:.4g}"
    if "SQ_ACTIVE_INST_VALU" in d and "SQ_WAVE_CYCLES" in d:
        extra += f" ACTIVE_INST_VALU/WAVE_CYCLES={d['SQ_ACTIVE_INST_VALU'] / d['SQ_WAVE_CYCLES']:.3f}"
    lines.append(f"{k}: grid={d['grid']} vgpr={d['vgpr']} agpr={d['agpr']} scratch/lane={d['scratch_per_lane']} "
                 f"lds={d['lds']} hbm_bytes={hbm if hbm is None else f'{hbm:.4g}'}" + extra)
with open(os.path.join(dst, f"{tag}_pmc_summary.txt"), "w") as f:
    f.write("\n".join(lines) + "\n")
with open(os.path.join(dst, f"{tag}_pmc_traffic.json"), "w") as f:
    json.dump(out, f, indent=1)
print("\n".join(lines))
