"""Summarise the stall-counter passes of tools/pmc_stall.sh into one text file.

Usage: python tools/summarize_stall.py <tag> [n]
Reads gpurun_out/stall_<tag>/p*/run_counter_collection.csv, averages each
counter over the dispatches of a kernel, and writes
profiles/<tag>_pmc_stall.txt: cycle-type counters as a share of
SQ_WAVE_CYCLES, instruction counters per wave.
"""
import csv
import glob
import hashlib
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHARE = ["SQ_ACTIVE_INST_VALU", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS"]
PERWAVE = ["SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_SALU", "SQ_IFETCH"]


def main():
    tag = sys.argv[1]
    n = sys.argv[2] if len(sys.argv) > 2 else "262144"
    vals = defaultdict(lambda: defaultdict(list))
    for path in sorted(glob.glob(os.path.join(ROOT, "gpurun_out", f"stall_{tag}", "p*", "run_counter_collection.csv"))):
        with open(path) as f:
            for row in csv.DictReader(f):
                k = row["Kernel_Name"].split("(")[0]
                vals[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    avg = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in vals.items()}
    sha = hashlib.sha256(open(os.path.join(ROOT, "cess_amd", "lib", "libcess_bls.so"), "rb").read()).hexdigest()
    lines = [f"# rocprofv3 stall counters, tag {tag} (tools/pmc_stall.sh, bench.py --n {n} --steps 1; "
             f"libcess_bls.so sha256 {sha})",
             "# per wave: share of SQ_WAVE_CYCLES; instruction counts per wave"]
    for k in sorted(avg):
        a = avg[k]
        waves = a.get("SQ_WAVES", 0.0)
        cyc = a.get("SQ_WAVE_CYCLES", 0.0)
        parts = [f"{k}: waves={waves:.0f}"]
        parts += [f"{c}={a[c] / cyc:.3f}" for c in SHARE if c in a and cyc]
        parts += [f"{c}/wave={a[c] / waves:.4g}" for c in PERWAVE if c in a and waves]
        lines.append(" ".join(parts))
    out = os.path.join(ROOT, "profiles", f"{tag}_pmc_stall.txt")
    with open(out, "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
