//! Node-side host functions for batch signature verification on MI355X
//!: the `sp_runtime_interface` the reference left
//! commented out at primitives/enclave-verify/src/lib.rs:10-14 and :35-44,
//! backed natively by the C ABI (include/cess_bls.h, include/cess_rsa.h)
//! through the `verify-bls-signatures-gpu` crate.
//!
//! UNCOMPILED HERE: this image has no cargo/rustc.  It is written against the
//! substrate crates the reference pins (Cargo.lock: sp-runtime-interface 7,
//! sp-externalities 0.13) and the C ABI this repository builds and tests.
//!
//! Consensus: a host function's result must not depend on the node's
//! hardware.  The GPU verdicts are bit-exact with the reference crate
//! (tests/test_gpu_parity.py, golden fixtures pinned by the reference KATs),
//! every infrastructure failure falls back to the reference crate on the CPU,
//! and a node without the extension registered runs the CPU path -- so every
//! node returns the same verdicts.
#![cfg_attr(not(feature = "std"), no_std)]

use sp_runtime_interface::runtime_interface;
use sp_std::vec::Vec;

/// Verdict codes of `verify_bls_batch` (include/cess_bls.h): 0 OK, 1 SIG_LEN,
/// 2 SIG_POINT, 3 PK_LEN, 4 PK_POINT, 5 PAIRING_FAIL.
pub const BLS_OK: u8 = 0;

#[cfg(feature = "std")]
pub mod ext {
    //! The externalities extension a node registers to route the host
    //! functions to a GPU (node/src/service.rs, patches/node_service.rs).
    use parking_lot::Mutex;
    use std::collections::HashMap;
    use std::sync::Arc;
    use verify_bls_signatures_gpu::{Config, Verifier};

    /// Shared GPU verifier plus a verdict cache that the node-side batcher
    /// (patches/node_batcher.rs) fills ahead of block execution: the runtime's
    /// per-extrinsic call then costs a hash lookup.
    pub struct GpuState {
        pub verifier: Mutex<Option<Verifier>>,
        pub cache: Mutex<HashMap<[u8; 32], u8>>,
    }

    impl GpuState {
        pub fn new(cfg: &Config) -> Arc<Self> {
            // no GPU / no library: the extension still works, on the CPU path
            Arc::new(GpuState { verifier: Mutex::new(Verifier::new(cfg).ok()), cache: Mutex::new(HashMap::new()) })
        }
    }

    sp_externalities::decl_extension! {
        /// Registered by the node; absent in wasm-only execution and tests.
        pub struct GpuVerifierExt(Arc<GpuState>);
    }

    /// Cache key of one record: blake2-256 over (sig, msg, key) with lengths.
    pub fn record_key(sig: &[u8], msg: &[u8], key: &[u8]) -> [u8; 32] {
        let mut buf = Vec::with_capacity(24 + sig.len() + msg.len() + key.len());
        for part in [sig, msg, key] {
            buf.extend_from_slice(&(part.len() as u64).to_le_bytes());
            buf.extend_from_slice(part);
        }
        sp_core_hashing::blake2_256(&buf)
    }

    /// The reference crate on the CPU: the fallback, and the semantics the GPU
    /// path reproduces (codes: signature first, then key, then pairing --
    /// utils/verify-bls-signatures/src/lib.rs:243-247).
    pub fn cpu_code(sig: &[u8], msg: &[u8], key: &[u8]) -> u8 {
        use ic_verify_bls_signature::{InvalidPublicKey, InvalidSignature, PublicKey, Signature};
        let s = match Signature::deserialize(sig) {
            Ok(s) => s,
            Err(InvalidSignature::WrongLength) => return 1,
            Err(_) => return 2,
        };
        let k = match PublicKey::deserialize(key) {
            Ok(k) => k,
            Err(InvalidPublicKey::WrongLength) => return 3,
            Err(_) => return 4,
        };
        if k.verify(msg, &s).is_ok() { 0 } else { 5 }
    }

    /// Codes for a batch: cache hits first, the rest in one GPU batch
    /// (cess_bls_verify_batch_var), the CPU if the GPU is absent or fails.
    pub fn batch_codes(st: &GpuState, sigs: &[Vec<u8>], msgs: &[Vec<u8>], keys: &[Vec<u8>]) -> Vec<u8> {
        let n = sigs.len();
        let mut codes = vec![u8::MAX; n];
        let mut miss = Vec::new();
        {
            let cache = st.cache.lock();
            for i in 0..n {
                match cache.get(&record_key(&sigs[i], &msgs[i], &keys[i])) {
                    Some(&c) => codes[i] = c,
                    None => miss.push(i),
                }
            }
        }
        if miss.is_empty() {
            return codes;
        }
        let recs: Vec<(&[u8], &[u8], &[u8])> =
            miss.iter().map(|&i| (&sigs[i][..], &msgs[i][..], &keys[i][..])).collect();
        let gpu = st.verifier.lock().as_mut().and_then(|v| v.verify_batch(&recs).ok());
        let mut cache = st.cache.lock();
        for (j, &i) in miss.iter().enumerate() {
            let c = match &gpu {
                Some(v) => v.codes[j],
                None => cpu_code(&sigs[i], &msgs[i], &keys[i]),
            };
            codes[i] = c;
            cache.insert(record_key(&sigs[i], &msgs[i], &keys[i]), c);
        }
        codes
    }
}

/// Host functions: `gpu_verify::verify_bls(..)` etc. in the runtime.
#[runtime_interface]
pub trait GpuVerify {
    /// `cp_enclave_verify::verify_bls(key, msg, sig)` (primitives/enclave-verify/
    /// src/lib.rs:230-235) without its panics: `None` where the reference
    /// unwraps a key or signature that does not deserialize, else the verdict.
    fn verify_bls(&mut self, key: &[u8], msg: &[u8], sig: &[u8]) -> Option<bool> {
        let code = self.verify_bls_batch(vec![sig.to_vec()], vec![msg.to_vec()], vec![key.to_vec()])[0];
        match code {
            0 => Some(true),
            5 => Some(false),
            _ => None,
        }
    }

    /// Batch form for node-side callers: one verdict code per record
    /// (sigs[i], msgs[i], keys[i]), codes as in include/cess_bls.h.
    fn verify_bls_batch(&mut self, sigs: Vec<Vec<u8>>, msgs: Vec<Vec<u8>>, keys: Vec<Vec<u8>>) -> Vec<u8> {
        assert!(sigs.len() == msgs.len() && msgs.len() == keys.len());
        match self.extension::<ext::GpuVerifierExt>() {
            Some(e) => ext::batch_codes(&e.0, &sigs, &msgs, &keys),
            None => (0..sigs.len()).map(|i| ext::cpu_code(&sigs[i], &msgs[i], &keys[i])).collect(),
        }
    }

    /// `cp_enclave_verify::verify_rsa(key, msg, sig)` (primitives/enclave-verify/
    /// src/lib.rs:221-228) without its panic: `None` where the SPKI key does
    /// not parse.  Podr2 checks are single calls; the GPU batch form is
    /// `Verifier::verify_rsa_batch` for node-side batchers.
    fn verify_rsa(&mut self, key: &[u8], msg: &[u8], sig: &[u8]) -> Option<bool> {
        if let Some(e) = self.extension::<ext::GpuVerifierExt>() {
            if let Some(v) = e.0.verifier.lock().as_mut() {
                match v.verify_rsa(key, msg, sig) {
                    Ok(ok) => return Some(ok),
                    Err(verify_bls_signatures_gpu::Error::BadKey) => return None,
                    Err(_) => {}   // infrastructure: fall through to the CPU
                }
            }
        }
        use rsa::{pkcs8::DecodePublicKey, Pkcs1v15Sign, PublicKey, RsaPublicKey};
        let pk = RsaPublicKey::from_public_key_der(key).ok()?;
        Some(pk.verify(Pkcs1v15Sign::new_raw(), msg, sig).is_ok())
    }
}
