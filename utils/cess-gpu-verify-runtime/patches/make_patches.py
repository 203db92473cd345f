"""Generate cess-gpu-verify.patch: the node / runtime / pallet wiring of the
MI355X batch verifier as ONE unified diff against
the reference tree, with no elisions.

The edits below are anchored on exact text of the reference files; each
anchor must occur exactly once, so a changed reference fails here instead of
producing a patch that does not apply.  Development tool: it reads
/root/reference (run it where that tree exists); the committed patch is the
product, checked by tests/test_patches.py with `git apply --check`.

    python utils/cess-gpu-verify-runtime/patches/make_patches.py [REFERENCE_ROOT]

The patch changes (file: what):
  Cargo.toml                          workspace members += the two utils crates
  primitives/common/src/lib.rs        TeeBlsSignature = [u8; 48], TeeBlsPublicKey = [u8; 96]
  c-pallets/tee-worker/src/lib.rs     TeeBlsKey storage, register_bls_key call (the key must deserialize
                                      as the reference crate's PublicKey: InvalidBlsKey otherwise), key
                                      removed on exit, ScheduleFind::bls_key (default None: other
                                      implementors unchanged)
  c-pallets/tee-worker/Cargo.toml     dependency on ic-verify-bls-signature (the reference crate)
  c-pallets/audit/src/lib.rs          submit_verify_result verifies the TEE worker's BLS signature over
                                      the verdict (was `_tee_signature: NodeSignature`, unchecked,
                                      "TODO! Podr2Key verify" at :480-484) with the non-panicking
                                      runtime::verify_bls_signature; weight += WASM_VERIFY_BLS_WEIGHT;
                                      verify_record / verify_result_message
  c-pallets/audit/Cargo.toml          dependency on cess-gpu-verify-runtime
  runtime/src/lib.rs                  spec_version / transaction_version bump (the call's encoding
                                      changes), decode_verify_record, GpuVerifyRecords runtime API
  runtime/Cargo.toml                  dependency on cess-gpu-verify-runtime
  node/src/executor.rs                ExtendHostFunctions += gpu_verify host functions
  node/src/service.rs                 GPU state, extensions factory and batcher task in new_partial
  node/src/main.rs, node/Cargo.toml   the gpu_batcher module (new file node/src/gpu_batcher.rs) and deps
"""
import os
import shutil
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.environ.get("CESS_PATCH_OUT") or os.path.join(HERE, "cess-gpu-verify.patch")
SUBSTRATE = 'git = "https://github.com/CESSProject/substrate.git", branch = "cess-polkadot-v0.9.36"'


def edit(text, old, new, path):
    n = text.count(old)
    if n != 1:
        raise SystemExit(f"{path}: anchor found {n} times: {old[:70]!r}")
    return text.replace(old, new)


EDITS = {
    "Cargo.toml": [
        ("    'primitives/*'\n]",
         "    'primitives/*',\n    'utils/verify-bls-signatures-gpu',\n    'utils/cess-gpu-verify-runtime',\n]"),
    ],
    "primitives/common/src/lib.rs": [
        ("pub type NodeSignature = [u8; 64];\n",
         "pub type NodeSignature = [u8; 64];\n"
         "/// A TEE worker's BLS12-381 verdict signature (compressed G1) and public key\n"
         "/// (compressed G2): the encodings of utils/verify-bls-signatures.\n"
         "pub type TeeBlsSignature = [u8; 48];\n"
         "pub type TeeBlsPublicKey = [u8; 96];\n"),
    ],
    "c-pallets/tee-worker/src/lib.rs": [
        ("\t\tVerifyCertFailed,\n\t}\n",
         "\t\tVerifyCertFailed,\n"
         "\t\t//register_bls_key: the key is not a compressed point of G2\n"
         "\t\tInvalidBlsKey,\n\t}\n"),
        ("\t\tUpdatePeerId { acc: AccountOf<T> },\n",
         "\t\tUpdatePeerId { acc: AccountOf<T> },\n\n\t\tRegisterBlsKey { acc: AccountOf<T> },\n"),
        ("\tpub(super) type TeePodr2Pk<T: Config> = StorageValue<_, Podr2Key>;\n",
         "\tpub(super) type TeePodr2Pk<T: Config> = StorageValue<_, Podr2Key>;\n\n"
         "\t/// The BLS12-381 key a TEE worker signs its audit verdicts with\n"
         "\t/// (pallet_audit::submit_verify_result checks the signature against it).\n"
         "\t#[pallet::storage]\n"
         "\t#[pallet::getter(fn tee_bls_key)]\n"
         "\tpub(super) type TeeBlsKey<T: Config> = StorageMap<_, Blake2_128Concat, AccountOf<T>, TeeBlsPublicKey>;\n"),
        ("\t\t\tTeeWorkerMap::<T>::remove(&sender);\n",
         "\t\t\tTeeWorkerMap::<T>::remove(&sender);\n\t\t\tTeeBlsKey::<T>::remove(&sender);\n"),
        ("\t\t\tSelf::deposit_event(Event::<T>::Exit { acc: sender });\n\n\t\t\tOk(())\n\t\t}\n",
         "\t\t\tSelf::deposit_event(Event::<T>::Exit { acc: sender });\n\n\t\t\tOk(())\n\t\t}\n\n"
         "\t\t/// Register (or replace) the caller's BLS12-381 verdict key: 96 bytes,\n"
         "\t\t/// a compressed G2 point as ic-verify-bls-signature's PublicKey.\n"
         "\t\t/// The key must deserialize as the reference crate's PublicKey\n"
         "\t\t/// (utils/verify-bls-signatures/src/lib.rs:68-82: a point of G2), so a\n"
         "\t\t/// stored key never makes a later verification fail on decoding.\n"
         "\t\t/// Weight: 10_000_000 for the storage work + 5_000_000_000 (5 ms), a\n"
         "\t\t/// conservative bound on one G2 decompression and subgroup check in\n"
         "\t\t/// wasm, until this call has a FRAME benchmark.\n"
         "\t\t#[pallet::call_index(9)]\n"
         "\t\t#[transactional]\n"
         "\t\t#[pallet::weight(10_000_000 + 5_000_000_000)]\n"
         "\t\tpub fn register_bls_key(origin: OriginFor<T>, key: TeeBlsPublicKey) -> DispatchResult {\n"
         "\t\t\tlet sender = ensure_signed(origin)?;\n"
         "\t\t\tensure!(TeeWorkerMap::<T>::contains_key(&sender), Error::<T>::NonTeeWorker);\n"
         "\t\t\tensure!(\n"
         "\t\t\t\tic_verify_bls_signature::PublicKey::deserialize(&key).is_ok(),\n"
         "\t\t\t\tError::<T>::InvalidBlsKey\n"
         "\t\t\t);\n"
         "\t\t\tTeeBlsKey::<T>::insert(&sender, key);\n"
         "\t\t\tSelf::deposit_event(Event::<T>::RegisterBlsKey { acc: sender });\n"
         "\t\t\tOk(())\n"
         "\t\t}\n"),
        ("\tfn get_controller_list() -> Vec<AccountId>;\n}\n",
         "\tfn get_controller_list() -> Vec<AccountId>;\n"
         "\t/// The TEE worker's registered BLS12-381 verdict key, if any.\n"
         "\tfn bls_key(_acc: &AccountId) -> Option<TeeBlsPublicKey> {\n"
         "\t\tNone\n"
         "\t}\n}\n"),
        ("\t\tacc_list\n\t}\n}\n",
         "\t\tacc_list\n\t}\n\n"
         "\tfn bls_key(acc: &AccountOf<T>) -> Option<TeeBlsPublicKey> {\n"
         "\t\tTeeBlsKey::<T>::get(acc)\n"
         "\t}\n}\n"),
    ],
    "c-pallets/tee-worker/Cargo.toml": [
        ("cp-enclave-verify = { path = '../../primitives/enclave-verify', version = '0.1.0', default-features = false }\n",
         "cp-enclave-verify = { path = '../../primitives/enclave-verify', version = '0.1.0', default-features = false }\n"
         "ic-verify-bls-signature = { path = '../../utils/verify-bls-signatures', version = '0.2.0', default-features = false }\n"),
    ],
    "c-pallets/audit/src/lib.rs": [
        ("\t\tNonExistentMission,\n\n\t\tUnexpectedError,\n",
         "\t\tNonExistentMission,\n\n\t\tUnexpectedError,\n"
         "\t\t//The TEE worker has no registered BLS key (pallet_tee_worker::register_bls_key)\n"
         "\t\tNoTeeBlsKey,\n"
         "\t\t//The TEE worker's signature over the verdict does not verify\n"
         "\t\tVerifyTeeSigFailed,\n"),
        ("\t\t#[pallet::weight(100_000_000)]\n\t\tpub fn submit_verify_result(",
         "\t\t// Weight: the reference's 100_000_000 plus a conservative bound on the\n"
         "\t\t// wasm BLS verification a node without a GPU verdict runs\n"
         "\t\t// (cess_gpu_verify_runtime::WASM_VERIFY_BLS_WEIGHT), until this call has\n"
         "\t\t// a FRAME benchmark with a signed verdict.\n"
         "\t\t#[pallet::weight(100_000_000 + cess_gpu_verify_runtime::WASM_VERIFY_BLS_WEIGHT)]\n"
         "\t\tpub fn submit_verify_result("),
        ("\t\t\t_tee_signature: NodeSignature,\n", "\t\t\ttee_signature: TeeBlsSignature,\n"),
        ("\t\t\t// TODO! Podr2Key verify\n",
         "\t\t\t// The TEE worker's BLS12-381 signature over the verdict and the\n"
         "\t\t\t// challenge round it answers, with the total semantics of\n"
         "\t\t\t// ic_verify_bls_signature::verify_bls_signature (a signature or key\n"
         "\t\t\t// that does not deserialize is an Err, never a panic): the MI355X\n"
         "\t\t\t// batch verifier's host function answers from its verdict cache, and\n"
         "\t\t\t// a node without a GPU verdict runs that reference function in wasm,\n"
         "\t\t\t// so every node reaches the same verdict.\n"
         "\t\t\tlet (sig, msg, key) =\n"
         "\t\t\t\tSelf::verify_record(&sender, &miner, idle_result, service_result, &tee_signature)\n"
         "\t\t\t\t\t.ok_or(Error::<T>::NoTeeBlsKey)?;\n"
         "\t\t\tensure!(\n"
         "\t\t\t\tcess_gpu_verify_runtime::runtime::verify_bls_signature(&sig, &msg, &key).is_ok(),\n"
         "\t\t\t\tError::<T>::VerifyTeeSigFailed\n"
         "\t\t\t);\n"),
        ("\timpl<T: Config> Pallet<T> {\n\t\tfn clear_challenge(",
         "\timpl<T: Config> Pallet<T> {\n"
         "\t\t/// The message a TEE worker signs for `submit_verify_result`: the SCALE\n"
         "\t\t/// encoding of the verdict and the challenge round it answers, so a\n"
         "\t\t/// signature cannot be replayed for another miner or round.\n"
         "\t\tpub fn verify_result_message(\n"
         "\t\t\tminer: &AccountOf<T>,\n"
         "\t\t\tidle_result: bool,\n"
         "\t\t\tservice_result: bool,\n"
         "\t\t\tstart: BlockNumberOf<T>,\n"
         "\t\t) -> Vec<u8> {\n"
         "\t\t\t(b\"cess/audit/verify-result\", miner, idle_result, service_result, start).encode()\n"
         "\t\t}\n\n"
         "\t\t/// The (signature, message, key) record `submit_verify_result` sent by\n"
         "\t\t/// `sender` verifies, built from the current state (also what the node's\n"
         "\t\t/// GPU batcher asks the runtime for, ahead of block execution); None\n"
         "\t\t/// without a registered key or a challenge snapshot.\n"
         "\t\tpub fn verify_record(\n"
         "\t\t\tsender: &AccountOf<T>,\n"
         "\t\t\tminer: &AccountOf<T>,\n"
         "\t\t\tidle_result: bool,\n"
         "\t\t\tservice_result: bool,\n"
         "\t\t\ttee_signature: &TeeBlsSignature,\n"
         "\t\t) -> Option<(Vec<u8>, Vec<u8>, Vec<u8>)> {\n"
         "\t\t\tlet key = T::Scheduler::bls_key(sender)?;\n"
         "\t\t\tlet snap_shot = <ChallengeSnapShot<T>>::try_get().ok()?;\n"
         "\t\t\tlet msg =\n"
         "\t\t\t\tSelf::verify_result_message(miner, idle_result, service_result, snap_shot.net_snap_shot.start);\n"
         "\t\t\tSome((tee_signature.to_vec(), msg, key.to_vec()))\n"
         "\t\t}\n\n"
         "\t\tfn clear_challenge("),
    ],
    "c-pallets/audit/Cargo.toml": [
        ("pallet-cess-staking = { path = '../staking', version = '4.0.0-dev', default-features = false }\n",
         "pallet-cess-staking = { path = '../staking', version = '4.0.0-dev', default-features = false }\n"
         "cess-gpu-verify-runtime = { path = '../../utils/cess-gpu-verify-runtime', default-features = false }\n"),
        ('\t"pallet-tee-worker/std",\n', '\t"pallet-tee-worker/std",\n\t"cess-gpu-verify-runtime/std",\n'),
    ],
    "runtime/Cargo.toml": [
        ("cp-enclave-verify = { path = '../primitives/enclave-verify', version = '0.1.0', default-features = false }\n",
         "cp-enclave-verify = { path = '../primitives/enclave-verify', version = '0.1.0', default-features = false }\n"
         "cess-gpu-verify-runtime = { path = '../utils/cess-gpu-verify-runtime', default-features = false }\n"),
        ('    "cp-enclave-verify/std",\n', '    "cp-enclave-verify/std",\n    "cess-gpu-verify-runtime/std",\n'),
    ],
    "runtime/src/lib.rs": [
        ("\tspec_version: 107,\n", "\tspec_version: 108,\n"),
        ("\ttransaction_version: 1,\n", "\ttransaction_version: 2,\n"),
        ("impl_runtime_apis! {\n",
         "/// The GPU batcher's question (runtime API\n"
         "/// cess_gpu_verify_runtime::GpuVerifyRecords): for a signed\n"
         "/// Audit::submit_verify_result, the (signature, message, key) record its\n"
         "/// dispatch will verify; nothing for other calls.\n"
         "pub fn decode_verify_record(xt: &UncheckedExtrinsic) -> Option<(Vec<u8>, Vec<u8>, Vec<u8>)> {\n"
         "\tlet (address, _, _) = xt.0.signature.as_ref()?;\n"
         "\tlet sender = <Runtime as frame_system::Config>::Lookup::lookup(address.clone()).ok()?;\n"
         "\tmatch &xt.0.function {\n"
         "\t\tRuntimeCall::Audit(pallet_audit::Call::submit_verify_result {\n"
         "\t\t\tminer,\n"
         "\t\t\tidle_result,\n"
         "\t\t\tservice_result,\n"
         "\t\t\ttee_signature,\n"
         "\t\t}) => pallet_audit::Pallet::<Runtime>::verify_record(\n"
         "\t\t\t&sender,\n"
         "\t\t\tminer,\n"
         "\t\t\t*idle_result,\n"
         "\t\t\t*service_result,\n"
         "\t\t\ttee_signature,\n"
         "\t\t),\n"
         "\t\t_ => None,\n"
         "\t}\n"
         "}\n\n"
         "impl_runtime_apis! {\n"
         "\timpl cess_gpu_verify_runtime::GpuVerifyRecords<Block> for Runtime {\n"
         "\t\tfn verify_records(xts: Vec<<Block as BlockT>::Extrinsic>) -> Vec<(Vec<u8>, Vec<u8>, Vec<u8>)> {\n"
         "\t\t\txts.iter().filter_map(decode_verify_record).collect()\n"
         "\t\t}\n"
         "\t}\n\n"),
    ],
    "node/src/executor.rs": [
        ("\ttype ExtendHostFunctions = frame_benchmarking::benchmarking::HostFunctions;\n",
         "\ttype ExtendHostFunctions = (\n"
         "\t\tframe_benchmarking::benchmarking::HostFunctions,\n"
         "\t\tcess_gpu_verify_runtime::gpu_verify::HostFunctions,\n"
         "\t);\n"),
    ],
    "node/src/main.rs": [
        ("mod executor;\n", "mod executor;\nmod gpu_batcher;\n"),
    ],
    "node/src/service.rs": [
        ("\t\tclient.clone(),\n\t);\n\tlet justification_import = grandpa_block_import.clone();\n",
         "\t\tclient.clone(),\n\t);\n\n"
         "\t// MI355X batch verifier: the gpu_verify host functions answer from the\n"
         "\t// GPU's verdict cache, filled ahead of execution by the batcher.  Without\n"
         "\t// a device every answer is UNAVAILABLE and the runtime's own verifier\n"
         "\t// runs, so consensus does not depend on the node's hardware.\n"
         "\tif let Some(gpu) = cess_gpu_verify_runtime::ext::GpuState::new(&Default::default()) {\n"
         "\t\tclient\n"
         "\t\t\t.execution_extensions()\n"
         "\t\t\t.set_extensions_factory(Box::new(crate::gpu_batcher::GpuExtensionsFactory(gpu.clone())));\n"
         "\t\ttask_manager.spawn_handle().spawn_blocking(\n"
         "\t\t\t\"gpu-verify-batcher\",\n"
         "\t\t\tNone,\n"
         "\t\t\tcrate::gpu_batcher::run(transaction_pool.clone(), client.clone(), gpu),\n"
         "\t\t);\n"
         "\t}\n\n"
         "\tlet justification_import = grandpa_block_import.clone();\n"),
    ],
    "node/Cargo.toml": [
        ("cess-node-runtime = { path = \"../runtime\" }\n",
         "cess-node-runtime = { path = \"../runtime\" }\n"
         "cess-gpu-verify-runtime = { path = \"../utils/cess-gpu-verify-runtime\" }\n"
         "ic-verify-bls-signature-gpu = { path = \"../utils/verify-bls-signatures-gpu\" }\n"
         f"sp-externalities = {{ version = \"0.13.0\", {SUBSTRATE} }}\n"),
    ],
}
NEW_FILES = {"node/src/gpu_batcher.rs": os.path.join(HERE, "gpu_batcher.rs")}


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    with tempfile.TemporaryDirectory() as tmp:
        git = ["git", "-C", tmp, "-c", "user.name=gen", "-c", "user.email=gen@localhost"]
        subprocess.check_call(git + ["init", "-q"])
        for rel in EDITS:
            dst = os.path.join(tmp, rel)
            os.makedirs(os.path.dirname(dst), exist_ok=True)
            shutil.copyfile(os.path.join(ref, rel), dst)
        subprocess.check_call(git + ["add", "-A"])
        subprocess.check_call(git + ["commit", "-qm", "reference"])
        for rel, eds in EDITS.items():
            p = os.path.join(tmp, rel)
            with open(p) as f:
                text = f.read()
            for old, new in eds:
                text = edit(text, old, new, rel)
            with open(p, "w") as f:
                f.write(text)
        for rel, src in NEW_FILES.items():
            assert not os.path.exists(os.path.join(ref, rel)), rel
            shutil.copyfile(src, os.path.join(tmp, rel))
        subprocess.check_call(git + ["add", "-A"])
        diff = subprocess.check_output(git + ["diff", "--cached", "--no-color", "--no-renames"])
    with open(OUT, "wb") as f:
        f.write(diff)
    print(OUT, len(diff), "bytes")


if __name__ == "__main__":
    main()
