// UNCOMPILED SKETCH (no cargo here): wiring the TEE verdict signature of
// c-pallets/audit to the gpu_verify host functions.
//
// Reference state: submit_verify_result takes `_tee_signature: NodeSignature`
// and never checks it (c-pallets/audit/src/lib.rs:480, "TODO! Podr2Key verify"
// at :484); NodeSignature = [u8; 64] (primitives/common/src/lib.rs:74) cannot
// hold a 48-byte BLS12-381 signature, and the tee-worker's BLS check is
// commented out (c-pallets/tee-worker/src/lib.rs:235-250).

// --- primitives/common/src/lib.rs ---------------------------------------------
/// A TEE worker's BLS12-381 verdict signature (compressed G1, 48 bytes) and
/// public key (compressed G2, 96 bytes), as in utils/verify-bls-signatures.
pub type TeeBlsSignature = [u8; 48];
pub type TeeBlsPublicKey = [u8; 96];

// --- c-pallets/tee-worker: the key a worker registers --------------------------
#[pallet::storage]
pub(super) type TeeBlsKey<T: Config> = StorageMap<_, Blake2_128Concat, AccountOf<T>, TeeBlsPublicKey>;

// --- c-pallets/audit/src/lib.rs ------------------------------------------------
/// The signed message: SCALE encoding of the verdict and the challenge it
/// answers, so a signature cannot be replayed for another miner or round.
pub fn verify_result_message<T: Config>(
    miner: &AccountOf<T>, idle_result: bool, service_result: bool, start: BlockNumberOf<T>,
) -> Vec<u8> {
    (b"cess/audit/verify-result", miner, idle_result, service_result, start).encode()
}

#[pallet::call_index(2)]
#[transactional]
#[pallet::weight(100_000_000)]
pub fn submit_verify_result(
    origin: OriginFor<T>,
    miner: AccountOf<T>,
    idle_result: bool,
    service_result: bool,
    tee_signature: TeeBlsSignature,
) -> DispatchResult {
    let sender = ensure_signed(origin)?;
    let key = T::TeeWorkerHandler::bls_key(&sender).ok_or(Error::<T>::NonExistentMission)?;
    let snap_shot = <ChallengeSnapShot<T>>::try_get().map_err(|_| Error::<T>::UnexpectedError)?;
    let msg = verify_result_message::<T>(&miner, idle_result, service_result, snap_shot.net_snap_shot.start);
    // host function: GPU batch verdict from the batcher's cache, a single GPU
    // call, or the reference crate on the CPU -- identical verdicts everywhere
    ensure!(
        cess_gpu_verify_runtime::gpu_verify::verify_bls(&key, &msg, &tee_signature) == Some(true),
        Error::<T>::VerifyTeeSigFailed
    );
    // ... the reference body from here on (reward / punish / remove), unchanged
    Ok(())
}
