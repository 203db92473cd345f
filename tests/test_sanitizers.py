"""CPU: AddressSanitizer + UndefinedBehaviorSanitizer over the host-emulation
build of the device arithmetic (tests/hostemu/emu.cpp: the kernels' headers
compiled for the host with -DCESS_HOSTEMU).  GPU sanitizers are not available
on the GPU pool, so the host build is where out-of-bounds limb indexing,
signed-overflow and shift UB in the shared headers are caught.  The driver
(tests/hostemu/san_main.cpp) checks the golden verdict codes of every
fixed-length record and that the staged and value-based pairing paths give the
same Gt bytes."""
import json
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HE = os.path.join(ROOT, "tests", "hostemu")


def test_hostemu_asan_ubsan(tmp_path):
    exe = str(tmp_path / "san_emu")
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-DCESS_HOSTEMU",
                           "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                           os.path.join(HE, "emu.cpp"), os.path.join(HE, "san_main.cpp"), "-o", exe])
    with open(os.path.join(ROOT, "tests", "golden", "vectors.json")) as f:
        v = json.load(f)
    cases = [c for c in v["cases"] if len(c["sig"]) == 96 and len(c["pk"]) == 192][:40]
    recs = tmp_path / "records.txt"
    recs.write_text("".join(f"{c['sig']} {c['msg'] or '-'} {c['pk']} {c['code']}\n" for c in cases))
    env = dict(os.environ, ASAN_OPTIONS="halt_on_error=1:detect_leaks=1", UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([exe, str(recs)], capture_output=True, text=True, timeout=900, env=env)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    assert f"OK: {len(cases)} records, 0 mismatches" in r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr
