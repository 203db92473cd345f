// UNCOMPILED (no cargo here) -- wiring the TEE verdict signature of
// c-pallets/audit to the gpu_verify host functions,
// and the runtime side of the node batcher (`decode_verify_record`).
//
// Reference state: submit_verify_result takes `_tee_signature: NodeSignature`
// and never checks it (c-pallets/audit/src/lib.rs:480, "TODO! Podr2Key verify"
// at :484); NodeSignature = [u8; 64] (primitives/common/src/lib.rs:74) cannot
// hold a 48-byte BLS12-381 signature, and the tee-worker's BLS check is
// commented out (c-pallets/tee-worker/src/lib.rs:235-250).
//
// MIGRATION AND WEIGHT (the extrinsic's encoding changes):
//  * `tee_signature` becomes TeeBlsSignature = [u8; 48]: the call's SCALE
//    encoding changes, so the runtime upgrade bumps `spec_version` AND
//    `transaction_version` (runtime/src/lib.rs VERSION); TEE workers must
//    upgrade their signer before the upgrade is enacted -- in-flight
//    transactions with a 64-byte signature fail to decode and are dropped from
//    the pool, nothing is stored, so no storage migration is needed for the
//    call.  TeeBlsKey is a NEW storage map (empty at the upgrade): workers
//    register their 96-byte BLS key with tee_worker::register_bls_key before
//    their verdicts are accepted (NonExistentMission until then).
//  * The declared weight must cover the slowest node, i.e. one without a GPU,
//    which runs the reference verifier in wasm (two pairings): re-run the FRAME
//    benchmark of submit_verify_result with a signed verdict and add that cost
//    to the current 100_000_000; the GPU node's lookup is cheaper, never
//    dearer, so no node is under-charged.

// --- primitives/common/src/lib.rs ---------------------------------------------
/// A TEE worker's BLS12-381 verdict signature (compressed G1, 48 bytes) and
/// public key (compressed G2, 96 bytes), as in utils/verify-bls-signatures.
pub type TeeBlsSignature = [u8; 48];
pub type TeeBlsPublicKey = [u8; 96];

// --- c-pallets/tee-worker: the key a worker registers --------------------------
#[pallet::storage]
pub(super) type TeeBlsKey<T: Config> = StorageMap<_, Blake2_128Concat, AccountOf<T>, TeeBlsPublicKey>;

#[pallet::call_index(9)]
#[pallet::weight(10_000_000)]
pub fn register_bls_key(origin: OriginFor<T>, key: TeeBlsPublicKey) -> DispatchResult {
    let sender = ensure_signed(origin)?;
    ensure!(TeeWorkerMap::<T>::contains_key(&sender), Error::<T>::NonTeeWorker);
    TeeBlsKey::<T>::insert(&sender, key);
    Ok(())
}

impl<T: Config> TeeWorkerHandler<AccountOf<T>> for Pallet<T> {
    // ... the reference handler methods, unchanged, plus:
    fn bls_key(acc: &AccountOf<T>) -> Option<TeeBlsPublicKey> {
        TeeBlsKey::<T>::get(acc)
    }
}

// --- c-pallets/audit/src/lib.rs ------------------------------------------------
/// The signed message: SCALE encoding of the verdict and the challenge it
/// answers, so a signature cannot be replayed for another miner or round.
pub fn verify_result_message<T: Config>(
    miner: &AccountOf<T>, idle_result: bool, service_result: bool, start: BlockNumberOf<T>,
) -> Vec<u8> {
    (b"cess/audit/verify-result", miner, idle_result, service_result, start).encode()
}

/// The (signature, message, key) record that `submit_verify_result` sent by
/// `sender` will verify, built from the current state; None if the call is not
/// a verdict submission or its inputs are not in storage (the extrinsic would
/// fail before verifying anything).
pub fn verify_record<T: Config>(
    sender: &AccountOf<T>, miner: &AccountOf<T>, idle_result: bool, service_result: bool,
    tee_signature: &TeeBlsSignature,
) -> Option<(Vec<u8>, Vec<u8>, Vec<u8>)> {
    let key = T::TeeWorkerHandler::bls_key(sender)?;
    let snap_shot = <ChallengeSnapShot<T>>::get()?;
    let msg = verify_result_message::<T>(miner, idle_result, service_result, snap_shot.net_snap_shot.start);
    Some((tee_signature.to_vec(), msg, key.to_vec()))
}

#[pallet::call_index(2)]
#[transactional]
#[pallet::weight(100_000_000 /* + the benchmarked wasm BLS verification, see MIGRATION AND WEIGHT */)]
pub fn submit_verify_result(
    origin: OriginFor<T>,
    miner: AccountOf<T>,
    idle_result: bool,
    service_result: bool,
    tee_signature: TeeBlsSignature,
) -> DispatchResult {
    let sender = ensure_signed(origin)?;
    let (sig, msg, key) = verify_record::<T>(&sender, &miner, idle_result, service_result, &tee_signature)
        .ok_or(Error::<T>::NonExistentMission)?;
    // host function: the GPU verdict from the batcher's cache or one GPU call;
    // without one (no GPU, or a record the GPU cannot answer) the reference's
    // own cp_enclave_verify::verify_bls runs here, in the runtime
    ensure!(cess_gpu_verify_runtime::runtime::verify_bls(&key, &msg, &sig), Error::<T>::VerifyTeeSigFailed);
    // ... the reference body from here on (reward / punish / remove), unchanged
    Ok(())
}

// --- runtime/src/lib.rs --------------------------------------------------------
/// The batcher's question (runtime API GpuVerifyRecords, ../src/lib.rs): for
/// each pool transaction that is a signed `Audit::submit_verify_result`, the
/// record its dispatch will verify.  Unsigned or other calls give nothing.
pub fn decode_verify_record(xt: &UncheckedExtrinsic) -> Option<(Vec<u8>, Vec<u8>, Vec<u8>)> {
    let (address, _, _) = xt.signature.as_ref()?;
    let sender = <Runtime as frame_system::Config>::Lookup::lookup(address.clone()).ok()?;
    match &xt.function {
        RuntimeCall::Audit(pallet_audit::Call::submit_verify_result {
            miner, idle_result, service_result, tee_signature,
        }) => pallet_audit::verify_record::<Runtime>(&sender, miner, *idle_result, *service_result, tee_signature),
        _ => None,
    }
}

impl_runtime_apis! {
    // ... the reference's runtime APIs, unchanged, plus:
    impl cess_gpu_verify_runtime::GpuVerifyRecords<Block> for Runtime {
        fn verify_records(xts: Vec<<Block as BlockT>::Extrinsic>) -> Vec<(Vec<u8>, Vec<u8>, Vec<u8>)> {
            xts.iter().filter_map(decode_verify_record).collect()
        }
    }
}
