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


READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"


def _kernel_notes(tmp_path):
    """{kernel symbol: {.private_segment_fixed_size, .vgpr_spill_count, ...}} of
    every gfx950 code object bundled in the library (AMDGPU metadata notes)."""
    lib = str(tmp_path / "libcess_bls.so")
    shutil.copy(LIB, lib)
    subprocess.check_call([OBJDUMP, "--offloading", lib], cwd=tmp_path, stdout=subprocess.DEVNULL)
    out = {}
    for o in glob.glob(str(tmp_path / "libcess_bls.so.*gfx950")):
        notes = subprocess.run([READELF, "--notes", o], capture_output=True, text=True, check=True).stdout
        cur = None
        for line in notes.splitlines():
            s = line.strip().lstrip("- ").strip()
            if s.startswith(".name:"):
                cur = s.split(":", 1)[1].strip()
                out.setdefault(cur, {})
            elif cur and ":" in s and s.split(":", 1)[0] in (".private_segment_fixed_size", ".vgpr_spill_count"):
                k, v = s.split(":", 1)
                try:
                    out[cur][k] = int(v.strip())
                except ValueError:
                    pass
    return out


@pytest.mark.skipif(not (os.path.exists(OBJDUMP) and os.path.exists(READELF)), reason="llvm tools not in this image")
def test_staged_kernels_scratch_budget(tmp_path):
    """The lane-fresh store addressing (bls/staged.hpp lane_fresh) keeps the
    Miller loop free of scratch and k_final's spill below 1 KiB per lane
    (round 3: k_miller 72 -> 0 B, k_final 2,012 -> 800 B); a regression to
    per-access scratch reloads of the LDS / slot addresses shows up here."""
    if not os.path.exists(LIB):
        pytest.skip("library not built (run __graft_entry__.build())")
    notes = _kernel_notes(tmp_path)
    miller = [v for k, v in notes.items() if k.startswith("_Z8k_miller")]
    pair = [v for k, v in notes.items() if k.startswith("_Z9k_miller2")]
    final = [v for k, v in notes.items() if "k_final" in k]
    assert miller and pair and final, sorted(notes)
    assert miller[0].get(".private_segment_fixed_size") == 0, miller
    # the lane-pair Miller loops (bls/pair.hpp) at two waves per SIMD: 256
    # registers and no scratch once the line coefficients come back by value
    # and the per-lane load offsets stay opaque (152 B -> 0, k_miller_rr2
    # 256 B -> 0; k_miller 124.5 -> 121.5 ms)
    assert pair[0].get(".private_segment_fixed_size", 1 << 20) == 0, pair
    rr2 = [v for k, v in notes.items() if k.startswith("_Z12k_miller_rr2")]
    assert rr2 and rr2[0].get(".private_segment_fixed_size", 1 << 20) == 0, rr2
    # the lane-pair final exponentiation (bls/pair_fe.hpp): no scratch
    final2 = [v for k, v in notes.items() if k.startswith("_Z8k_final2")]
    assert final2 and final2[0].get(".private_segment_fixed_size", 1 << 20) <= 64, final2
    assert final[0].get(".private_segment_fixed_size", 1 << 20) <= 1024, final
    # the SSWU values parked in LDS (bls/h2c.hpp hash_to_g1_parked): k_hash and
    # k_hash_out 304 -> 24 B/lane, k_sign 512 -> 384 (its GLV ladder spills the
    # rest).  Round 6: the uniform-branch window lookup of
    # pow_fixed (CESS_POW_SWITCH) takes k_hash to 84 B -- every access outside
    # the loops, one spill and reload around each powering, and the kernel
    # 24.6 -> 24.3 ms (profiles/round6_an_sweep_pow_switch.txt)
    for name, cap in (("k_hash", 96), ("k_hash_out", 96), ("k_sign", 400)):
        ks = [v for k, v in notes.items() if k.startswith("_Z%d%s" % (len(name), name))]
        assert ks and ks[0].get(".private_segment_fixed_size", 1 << 20) <= cap, (name, ks)
