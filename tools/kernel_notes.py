"""Per-kernel register / scratch figures of the gfx950 code objects bundled in
cess_amd/lib/libcess_bls.so (AMDGPU metadata notes): .vgpr_count,
.agpr_count, .vgpr_spill_count, .private_segment_fixed_size (scratch bytes per
lane), .group_segment_fixed_size (LDS).  Usage: python tools/kernel_notes.py [name-filter]"""
import glob
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.environ.get("CESS_BLS_LIB") or os.path.join(ROOT, "cess_amd", "lib", "libcess_bls.so")
BIN = "/opt/rocm/lib/llvm/bin"
KEYS = (".vgpr_count", ".agpr_count", ".vgpr_spill_count", ".private_segment_fixed_size", ".group_segment_fixed_size")


def notes():
    out = {}
    with tempfile.TemporaryDirectory() as t:
        lib = os.path.join(t, "lib.so")
        shutil.copy(LIB, lib)
        subprocess.check_call([os.path.join(BIN, "llvm-objdump"), "--offloading", lib], cwd=t, stdout=subprocess.DEVNULL)
        for o in glob.glob(os.path.join(t, "lib.so.*gfx950")):
            txt = subprocess.run([os.path.join(BIN, "llvm-readelf"), "--notes", o], capture_output=True, text=True,
                                 check=True).stdout
            cur, vals = None, {}
            for line in txt.splitlines():
                s = line.strip().lstrip("- ").strip()
                k = s.split(":", 1)[0]
                if k in KEYS:
                    vals[k] = s.split(":", 1)[1].strip()
                elif k == ".name":
                    cur = s.split(":", 1)[1].strip()
                    out[cur] = vals
                if k == ".name":
                    pass
                if s.startswith(".wavefront_size"):
                    vals = {}
    return out


if __name__ == "__main__":
    flt = sys.argv[1] if len(sys.argv) > 1 else ""
    for k, v in sorted(notes().items()):
        if flt in k:
            print(f"{k:28s} " + " ".join(f"{kk.strip('.')}={v.get(kk, '-')}" for kk in KEYS))
