"""CPU: the shipped gfx950 code objects contain no device-function calls.

Round 1 hit a GPU hang with an out-of-line device function (k_rlc.hip's
mul128_w2).  tools/rlc_call_probe.hip reproduced it on MI355X and the ISA
showed the cause: in a callee longer than s_branch's reach, branch relaxation
routes long branches through s[30:31], the return-address pair, without
saving it, so the callee's return jumps to itself.  The product avoids the
hazard by having no callees (every device helper is __forceinline__); this
test disassembles every code object bundled in libcess_bls.so and fails if a
call (s_swappc_b64) appears, e.g. after a helper loses its force-inline."""
import glob
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "cess_amd", "lib", "libcess_bls.so")
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"


@pytest.mark.skipif(not os.path.exists(OBJDUMP), reason="llvm-objdump not in this image")
def test_no_device_calls_in_product(tmp_path):
    if not os.path.exists(LIB):
        pytest.skip("library not built (run __graft_entry__.build())")
    lib = str(tmp_path / "libcess_bls.so")
    shutil.copy(LIB, lib)
    subprocess.check_call([OBJDUMP, "--offloading", lib], cwd=tmp_path, stdout=subprocess.DEVNULL)
    objs = glob.glob(str(tmp_path / "libcess_bls.so.*gfx950"))
    assert objs, "no gfx950 code object bundled"
    kernels = 0
    for o in objs:
        dis = subprocess.run([OBJDUMP, "-d", o], capture_output=True, text=True, check=True).stdout
        assert "s_swappc_b64" not in dis, f"device call in {os.path.basename(o)}"
        kernels += dis.count(">:\n")
    assert kernels > 0
