//! Node-side host functions for batch signature verification on MI355X
//!: the `sp_runtime_interface` the reference left
//! commented out at primitives/enclave-verify/src/lib.rs:10-14 and :35-44,
//! backed natively by the C ABI (include/cess_bls.h, include/cess_rsa.h)
//! through the `ic-verify-bls-signature-gpu` crate.
//!
//! UNCOMPILED HERE: this image has no cargo/rustc.  It is written against the
//! substrate crates the reference pins (Cargo.lock: sp-runtime-interface 7,
//! sp-externalities 0.13, sp-api 4.0.0-dev) and the C ABI this repository
//! builds and tests.  The behaviour the host functions rely on -- the verdict
//! cache, its one-batch verification of misses and its "unavailable" answer --
//! is the C library's `cess_bls_cache_*`, tested through ctypes against the
//! golden codes (tests/test_service.py, CPU and MI355X).
//!
//! Consensus: a host function's answer must not depend on the node's hardware.
//! The host functions therefore carry NO verifier of their own besides the
//! GPU: every answer is either a GPU verdict (bit-exact with the reference
//! crate: tests/test_gpu_parity.py, fixtures pinned by the reference KATs) or
//! `UNAVAILABLE` (no extension, no device, an infrastructure failure, a key the
//! GPU cannot represent), on which the runtime runs the reference's own code
//! in wasm (`runtime::verify_bls_signature`, `runtime::verify_bls`,
//! `runtime::verify_rsa` below).  So every node reaches the reference's
//! verdict, and a node without a GPU simply executes the original wasm path.
//!
//! Where the node-side pieces live: the extensions factory, the host-function
//! registration and the batcher are hunks of patches/cess-gpu-verify.patch
//! (node/src/service.rs, node/src/executor.rs, and the new file
//! node/src/gpu_batcher.rs from patches/gpu_batcher.rs); the runtime side
//! (`decode_verify_record`, the audit call) is in the same patch.
#![cfg_attr(not(feature = "std"), no_std)]

use sp_runtime_interface::runtime_interface;
use sp_std::vec::Vec;

/// Answers of the single-record host functions.
pub const HOOK_FALSE: u8 = 0;
pub const HOOK_TRUE: u8 = 1;
/// No GPU verdict: the runtime's own verifier decides.
pub const HOOK_UNAVAILABLE: u8 = 0xff;

/// Verdict codes of `verify_bls_batch` (include/cess_bls.h): 0 OK, 1 SIG_LEN,
/// 2 SIG_POINT, 3 PK_LEN, 4 PK_POINT, 5 PAIRING_FAIL, 0xff UNAVAILABLE.
pub const BLS_OK: u8 = 0;
pub const BLS_SIG_LEN: u8 = 1;
pub const BLS_SIG_POINT: u8 = 2;
pub const BLS_PK_LEN: u8 = 3;
pub const BLS_PK_POINT: u8 = 4;
pub const BLS_PAIRING_FAIL: u8 = 5;
pub const BLS_UNAVAILABLE: u8 = 0xff;

/// Conservative weight (ref_time, picoseconds) of ONE
/// `ic_verify_bls_signature::verify_bls_signature` executed in wasm: hash to
/// G1, two Miller loops and a final exponentiation, ~3-5 ms natively for the
/// bls12_381 crate, taken x4 for wasm execution and rounded up to 20 ms.  A
/// call that may verify must declare at least this on top of its own weight:
/// a node without a GPU verdict runs exactly that wasm.  Replace it with the
/// call's FRAME benchmark (run with a signed verdict) when one exists.
pub const WASM_VERIFY_BLS_WEIGHT: u64 = 20_000_000_000;

#[cfg(feature = "std")]
pub mod ext {
    //! The externalities extension a node registers to route the host
    //! functions to a GPU (patches/cess-gpu-verify.patch: node/src/executor.rs
    //! and node/src/service.rs).
    use parking_lot::Mutex;
    use std::sync::Arc;
    use verify_bls_signatures_gpu::{Config, Error, VerdictCache, Verifier};

    /// Entries of the verdict cache: at ~100 B each, 1 M entries bound the
    /// cache to ~100 MB whatever the transaction pool receives.
    pub const CACHE_CAPACITY: usize = 1 << 20;

    /// The node's GPU verifier and the C library's bounded verdict cache,
    /// which the node-side batcher (node/src/gpu_batcher.rs, added by
    /// patches/cess-gpu-verify.patch from patches/gpu_batcher.rs) fills ahead
    /// of block execution: the runtime's per-extrinsic call is then a lookup.
    pub struct GpuState {
        pub verifier: Mutex<Option<Verifier>>,
        pub cache: VerdictCache,
    }

    impl GpuState {
        /// `None` if the cache cannot be created; a missing GPU is not an
        /// error (every lookup miss is then UNAVAILABLE: the runtime decides).
        pub fn new(cfg: &Config) -> Option<Arc<Self>> {
            let cache = VerdictCache::new(CACHE_CAPACITY).ok()?;
            Some(Arc::new(GpuState { verifier: Mutex::new(Verifier::new(cfg).ok()), cache }))
        }

        /// Codes for a batch of records: cached verdicts, the misses verified
        /// in one GPU batch (cess_bls_cache_verify_var) and cached; without a
        /// verifier, or when the batch fails, the misses are BLS_UNAVAILABLE
        /// and nothing is cached.
        pub fn batch_codes(&self, recs: &[(&[u8], &[u8], &[u8])]) -> Vec<u8> {
            let mut guard = self.verifier.lock();
            let (codes, _stats, _status) = self.cache.verify(guard.as_mut(), recs);
            codes
        }

        /// `cp_enclave_verify::verify_rsa` on the GPU: Some(verdict), or None
        /// (no device, infrastructure failure, a key the reference parses but
        /// the GPU cannot verify, a key that does not parse -- the runtime's
        /// own call then reproduces the reference, panic included).
        pub fn rsa(&self, key: &[u8], msg: &[u8], sig: &[u8]) -> Option<bool> {
            let mut guard = self.verifier.lock();
            match guard.as_mut()?.verify_rsa(key, msg, sig) {
                Ok(v) => Some(v),
                Err(Error::BadKey) | Err(Error::Unsupported) | Err(_) => None,
            }
        }
    }

    sp_externalities::decl_extension! {
        /// Registered by the node; absent in wasm-only execution and tests.
        pub struct GpuVerifierExt(Arc<GpuState>);
    }
}

/// Host functions: `gpu_verify::verify_bls(..)` etc. in the runtime.
#[runtime_interface]
pub trait GpuVerify {
    /// `cp_enclave_verify::verify_bls(key, msg, sig)` (primitives/enclave-verify/
    /// src/lib.rs:230-235) on the GPU: HOOK_TRUE / HOOK_FALSE for a verdict,
    /// HOOK_UNAVAILABLE otherwise -- including records the reference would
    /// panic on (key, then signature, not deserializing), so the panic stays
    /// the runtime's own.  (Callers that must not panic use
    /// `runtime::verify_bls_signature`, which reads the batch codes.)
    fn verify_bls(&mut self, key: &[u8], msg: &[u8], sig: &[u8]) -> u8 {
        let code = self.verify_bls_batch(vec![sig.to_vec()], vec![msg.to_vec()], vec![key.to_vec()])[0];
        match code {
            BLS_OK => HOOK_TRUE,
            BLS_PAIRING_FAIL => HOOK_FALSE,
            _ => HOOK_UNAVAILABLE,
        }
    }

    /// Batch form for node-side callers: one code per record (sigs[i],
    /// msgs[i], keys[i]), codes as in include/cess_bls.h, BLS_UNAVAILABLE
    /// without a GPU verdict.
    fn verify_bls_batch(&mut self, sigs: Vec<Vec<u8>>, msgs: Vec<Vec<u8>>, keys: Vec<Vec<u8>>) -> Vec<u8> {
        if sigs.len() != msgs.len() || msgs.len() != keys.len() {
            return sp_std::vec![BLS_UNAVAILABLE; sigs.len().max(msgs.len()).max(keys.len())];
        }
        match self.extension::<ext::GpuVerifierExt>() {
            Some(e) => {
                let recs: Vec<(&[u8], &[u8], &[u8])> =
                    (0..sigs.len()).map(|i| (&sigs[i][..], &msgs[i][..], &keys[i][..])).collect();
                e.0.batch_codes(&recs)
            }
            None => sp_std::vec![BLS_UNAVAILABLE; sigs.len()],
        }
    }

    /// `cp_enclave_verify::verify_rsa(key, msg, sig)` (primitives/enclave-verify/
    /// src/lib.rs:221-228) on the GPU: HOOK_TRUE / HOOK_FALSE, or
    /// HOOK_UNAVAILABLE (no GPU, a key the GPU cannot verify or parse).
    fn verify_rsa(&mut self, key: &[u8], msg: &[u8], sig: &[u8]) -> u8 {
        match self.extension::<ext::GpuVerifierExt>().and_then(|e| e.0.rsa(key, msg, sig)) {
            Some(true) => HOOK_TRUE,
            Some(false) => HOOK_FALSE,
            None => HOOK_UNAVAILABLE,
        }
    }
}

/// What the runtime calls (wasm and native alike): the GPU's verdict when the
/// node has one, else the reference's own code path, unchanged.  The
/// `cp-enclave-verify` and `ic-verify-bls-signature` dependencies here are the
/// runtime's existing wasm verifiers, not part of the node-side hook.
pub mod runtime {
    use super::*;

    /// Drop-in for `ic_verify_bls_signature::verify_bls_signature(sig, msg, key)
    /// -> Result<(), ()>` (utils/verify-bls-signatures/src/lib.rs:243-247): total,
    /// it never panics.  The GPU's codes are that function's own verdicts,
    /// bit-exact (tests/test_gpu_parity.py, tests/test_service.py): 0 is Ok, a
    /// signature or key that does not deserialize (codes 1-4, the reference's
    /// `map_err(|_| ())?` at :244-245) and a failed pairing check (5) are Err.
    /// Only BLS_UNAVAILABLE (no GPU verdict) runs the reference function itself,
    /// in wasm -- not `cp_enclave_verify::verify_bls`, which unwraps both
    /// deserialisations (primitives/enclave-verify/src/lib.rs:231, :233).
    pub fn verify_bls_signature(sig: &[u8], msg: &[u8], key: &[u8]) -> Result<(), ()> {
        let code = gpu_verify::verify_bls_batch(sp_std::vec![sig.to_vec()], sp_std::vec![msg.to_vec()], sp_std::vec![key.to_vec()]);
        match code.first().copied().unwrap_or(BLS_UNAVAILABLE) {
            BLS_OK => Ok(()),
            BLS_SIG_LEN | BLS_SIG_POINT | BLS_PK_LEN | BLS_PK_POINT | BLS_PAIRING_FAIL => Err(()),
            _ => ic_verify_bls_signature::verify_bls_signature(sig, msg, key),
        }
    }

    /// `ic_verify_bls_signature::PublicKey::deserialize(key).is_ok()`
    /// (utils/verify-bls-signatures/src/lib.rs:68-82): 96 bytes, a compressed
    /// point of G2.  What a pallet checks before it stores a key that later
    /// verifications will use.
    pub fn bls_public_key_is_valid(key: &[u8]) -> bool {
        ic_verify_bls_signature::PublicKey::deserialize(key).is_ok()
    }

    /// Drop-in for `cp_enclave_verify::verify_bls(key, msg, sig) -> Result<(), ()>`
    /// (primitives/enclave-verify/src/lib.rs:230): same signature AND the same
    /// panics (a key or signature that does not deserialize reaches the
    /// reference's unwrap), for the reference's existing call sites only.  New
    /// callers -- the audit wiring of patches/cess-gpu-verify.patch among them --
    /// use `verify_bls_signature` above.
    pub fn verify_bls(key: &[u8], msg: &[u8], sig: &[u8]) -> Result<(), ()> {
        match gpu_verify::verify_bls(key, msg, sig) {
            HOOK_TRUE => Ok(()),
            HOOK_FALSE => Err(()),
            _ => cp_enclave_verify::verify_bls(key, msg, sig),
        }
    }

    /// Drop-in for `cp_enclave_verify::verify_rsa(key, msg, sig)`.
    pub fn verify_rsa(key: &[u8], msg: &[u8], sig: &[u8]) -> bool {
        match gpu_verify::verify_rsa(key, msg, sig) {
            HOOK_TRUE => true,
            HOOK_FALSE => false,
            _ => cp_enclave_verify::verify_rsa(key, msg, sig),
        }
    }
}

sp_api::decl_runtime_apis! {
    /// What the node-side batcher asks the runtime (node/src/gpu_batcher.rs):
    /// the (signature, message, key) records that the given pool transactions
    /// will ask `gpu_verify::verify_bls_batch` about -- the runtime has the
    /// storage (TEE keys, challenge snapshot) to build them.  Implemented in the
    /// runtime by `decode_verify_record` (runtime/src/lib.rs hunk of
    /// patches/cess-gpu-verify.patch).
    pub trait GpuVerifyRecords {
        fn verify_records(xts: Vec<Block::Extrinsic>) -> Vec<(Vec<u8>, Vec<u8>, Vec<u8>)>;
    }
}
