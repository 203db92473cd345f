"""CPU: the node / runtime / pallet wiring is an
appliable patch against the reference tree, not a sketch.

* `utils/cess-gpu-verify-runtime/patches/cess-gpu-verify.patch` applies
  (`git apply --check`, then a real `git apply`) to a copy of /root/reference
  with the two utils crates of this repo added, and the patched files carry
  the wiring: the audit extrinsic verifies the TEE worker's BLS signature
  (reference: `_tee_signature: NodeSignature` unchecked, c-pallets/audit/src/
  lib.rs:480-484), the node registers the host functions (node/src/
  executor.rs:8) and the batcher.
* The committed patch equals what the generator (make_patches.py) produces
  from the reference today.
The Rust stays uncompiled (no cargo in this image).  Skipped where the
reference tree is absent (the GPU box).
"""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
PATCHES = os.path.join(ROOT, "utils", "cess-gpu-verify-runtime", "patches")
PATCH = os.path.join(PATCHES, "cess-gpu-verify.patch")

pytestmark = pytest.mark.skipif(not os.path.isdir(REF) or shutil.which("git") is None,
                                reason="reference tree or git absent")


@pytest.fixture(scope="module")
def tree(tmp_path_factory):
    t = tmp_path_factory.mktemp("ref") / "cess"
    shutil.copytree(REF, t, symlinks=True)
    for crate in ("cess-gpu-verify-runtime", "verify-bls-signatures-gpu"):
        assert not (t / "utils" / crate).exists()
        shutil.copytree(os.path.join(ROOT, "utils", crate), t / "utils" / crate)
    return t


def test_patch_applies(tree):
    subprocess.run(["git", "apply", "--check", "-p1", PATCH], cwd=tree, check=True, capture_output=True)
    subprocess.run(["git", "apply", "-p1", PATCH], cwd=tree, check=True, capture_output=True)
    audit = (tree / "c-pallets/audit/src/lib.rs").read_text()
    assert "tee_signature: TeeBlsSignature," in audit and "_tee_signature" not in audit
    # the verdict check is total: the non-panicking drop-in of the reference's
    # verify_bls_signature, never the unwrapping cp_enclave_verify::verify_bls
    # (primitives/enclave-verify/src/lib.rs:231, :233) nor the runtime::verify_bls
    # drop-in that falls back to it
    assert "cess_gpu_verify_runtime::runtime::verify_bls_signature(&sig, &msg, &key).is_ok()" in audit
    assert "runtime::verify_bls(" not in audit and "cp_enclave_verify::verify_bls" not in audit
    assert "unwrap()" not in _added(PATCH, "c-pallets/audit/src/lib.rs")
    assert "pub fn verify_record(" in audit
    # the call's weight covers the wasm verification a node without a GPU verdict runs
    assert "#[pallet::weight(100_000_000 + cess_gpu_verify_runtime::WASM_VERIFY_BLS_WEIGHT)]\n\t\tpub fn submit_verify_result(" in audit
    tee = (tree / "c-pallets/tee-worker/src/lib.rs").read_text()
    assert "pub fn register_bls_key(" in tee and "fn bls_key(" in tee
    # register_bls_key validates the key with the reference crate before storing it
    reg = tee[tee.index("pub fn register_bls_key("):]
    reg = reg[:reg.index("Ok(())")]
    assert reg.index("ic_verify_bls_signature::PublicKey::deserialize(&key).is_ok()") < reg.index("TeeBlsKey::<T>::insert")
    assert "Error::<T>::InvalidBlsKey" in reg and "\t\tInvalidBlsKey,\n" in tee
    assert "ic-verify-bls-signature = { path = '../../utils/verify-bls-signatures'" in \
        (tree / "c-pallets/tee-worker/Cargo.toml").read_text()
    assert "#[pallet::weight(10_000_000 + 5_000_000_000)]\n\t\tpub fn register_bls_key(" in tee
    assert "cess_gpu_verify_runtime::gpu_verify::HostFunctions" in (tree / "node/src/executor.rs").read_text()
    assert "GpuExtensionsFactory" in (tree / "node/src/service.rs").read_text()
    assert (tree / "node/src/gpu_batcher.rs").is_file()
    rt = (tree / "runtime/src/lib.rs").read_text()
    assert "impl cess_gpu_verify_runtime::GpuVerifyRecords<Block> for Runtime" in rt
    assert "pub type TeeBlsSignature = [u8; 48];" in (tree / "primitives/common/src/lib.rs").read_text()
    members = (tree / "Cargo.toml").read_text()
    assert "'utils/cess-gpu-verify-runtime'" in members and "'utils/verify-bls-signatures-gpu'" in members
    # no elided bodies anywhere in the patch
    body = open(PATCH).read()
    assert "unchanged" not in body.replace("consensus does not depend", "")
    assert "..." not in "".join(l for l in body.splitlines() if l.startswith("+"))


def _added(patch, path):
    """The '+' lines the patch adds to one file."""
    out, cur = [], None
    for line in open(patch).read().splitlines():
        if line.startswith("+++ "):
            cur = line[6:] if line.startswith("+++ b/") else None
        elif cur == path and line.startswith("+"):
            out.append(line[1:])
    return "\n".join(out)


def test_patch_is_generated(tmp_path):
    out = tmp_path / "gen.patch"
    subprocess.run([sys.executable, os.path.join(PATCHES, "make_patches.py"), REF], check=True,
                   env=dict(os.environ, CESS_PATCH_OUT=str(out)), capture_output=True)
    assert out.read_bytes() == open(PATCH, "rb").read()


def test_runtime_total_verify_maps_codes():
    """runtime::verify_bls_signature (what the audit wiring calls) is total:
    GPU codes 1-5 are Err directly, 0 is Ok, and ONLY an unavailable verdict
    falls back -- to the reference's non-panicking verify_bls_signature
    (utils/verify-bls-signatures/src/lib.rs:243-247), whose signature it keeps."""
    src = open(os.path.join(ROOT, "utils", "cess-gpu-verify-runtime", "src", "lib.rs")).read()
    ref = open(os.path.join(REF, "utils", "verify-bls-signatures", "src", "lib.rs")).read()
    assert "pub fn verify_bls_signature(sig: &[u8], msg: &[u8], key: &[u8]) -> Result<(), ()>" in ref
    body = src[src.index("pub fn verify_bls_signature(sig: &[u8], msg: &[u8], key: &[u8]) -> Result<(), ()> {"):]
    body = body[:body.index("\n    }\n")]
    assert "BLS_OK => Ok(())" in body
    assert "BLS_SIG_LEN | BLS_SIG_POINT | BLS_PK_LEN | BLS_PK_POINT | BLS_PAIRING_FAIL => Err(())" in body
    assert "_ => ic_verify_bls_signature::verify_bls_signature(sig, msg, key)" in body
    assert "cp_enclave_verify" not in body and "unwrap()" not in body
    # the codes are the C ABI's (include/cess_bls.h)
    hdr = open(os.path.join(ROOT, "include", "cess_bls.h")).read()
    for name, val in (("SIG_LEN", 1), ("SIG_POINT", 2), ("PK_LEN", 3), ("PK_POINT", 4), ("PAIRING_FAIL", 5)):
        assert f"pub const BLS_{name}: u8 = {val};" in src
        assert f"CESS_BLS_CODE_{name}" in hdr
    # no stale references to the deleted patch fragments
    for stale in ("patches/node.rs", "patches/node_batcher.rs", "patches/audit.rs"):
        assert stale not in src


def test_runtime_dropin_signature_matches_reference():
    """runtime::verify_bls has the reference's signature (cp_enclave_verify::
    verify_bls -> Result<(), ()>, primitives/enclave-verify/src/lib.rs:230), so
    its fallback arm type-checks and reference call sites take it unchanged."""
    src = open(os.path.join(ROOT, "utils", "cess-gpu-verify-runtime", "src", "lib.rs")).read()
    ref = open(os.path.join(REF, "primitives", "enclave-verify", "src", "lib.rs")).read()
    assert "pub fn verify_bls(key: &[u8], msg: &[u8], sig: &[u8]) -> Result<(), ()>" in ref
    assert "pub fn verify_bls(key: &[u8], msg: &[u8], sig: &[u8]) -> Result<(), ()> {" in src
    assert "pub fn verify_rsa(key: &[u8], msg: &[u8], sig: &[u8]) -> bool" in ref
    assert "pub fn verify_rsa(key: &[u8], msg: &[u8], sig: &[u8]) -> bool {" in src
