"""The C ABI through a C compiler: tests/c/cabi_golden.c is compiled by gcc as
strict C99 against include/cess_bls.h and linked with libcess_bls.so.

CPU: it compiles warning-free and, without a GPU, ctx_create fails loudly
(exit 2 = CESS_BLS_E_NO_DEVICE: there is no CPU fallback).
GPU: it verifies every golden record (tests/golden/vectors.json, oracle codes)
through cess_bls_verify_batch_var, cess_bls_verify and cess_bls_verify_batch."""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "cess_amd", "lib")


def _build(tmp_path):
    exe = str(tmp_path / "cabi_golden")
    subprocess.check_call(["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", "-pedantic", "-O1",
                           "-I", os.path.join(ROOT, "include"), os.path.join(ROOT, "tests", "c", "cabi_golden.c"),
                           "-L", LIBDIR, "-lcess_bls", "-Wl,-rpath," + LIBDIR, "-o", exe])
    return exe


def _records(tmp_path, with_lengths=True):
    with open(os.path.join(ROOT, "tests", "golden", "vectors.json")) as f:
        v = json.load(f)
    cases = v["cases"] + (v["length_cases"] if with_lengths else [])
    p = tmp_path / "records.txt"
    with open(p, "w") as f:
        for c in cases:
            f.write(f"{c['sig'] or '-'} {c['msg'] or '-'} {c['pk'] or '-'} {c['code']}\n")
    return str(p), len(cases)


def _run(exe, recs):
    env = dict(os.environ)
    env.pop("LD_LIBRARY_PATH", None)
    return subprocess.run([exe, recs], capture_output=True, text=True, timeout=300, env=env)


def test_c_compiles_and_fails_loudly_without_gpu(tmp_path):
    import torch
    exe = _build(tmp_path)
    if torch.cuda.device_count() > 0:
        pytest.skip("GPU present (the -m gpu test runs the program)")
    recs, _ = _records(tmp_path)
    r = _run(exe, recs)
    assert r.returncode == 2, (r.returncode, r.stdout, r.stderr)
    assert "CPU fallback" in r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("with_lengths", [True, False])
def test_c_program_golden_codes(tmp_path, with_lengths):
    exe = _build(tmp_path)
    recs, n = _records(tmp_path, with_lengths)
    r = _run(exe, recs)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
    assert f"OK: {n} records, 0 mismatches" in r.stdout
