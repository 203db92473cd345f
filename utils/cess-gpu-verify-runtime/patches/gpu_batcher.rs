//! Node-side batcher and externalities wiring of the MI355X batch verifier
//!.  UNCOMPILED here (no cargo in this image);
//! written against the substrate branch the reference node pins
//! (node/Cargo.toml: cess-polkadot-v0.9.36).
//!
//! * `GpuExtensionsFactory` attaches the GPU state to every runtime call the
//!   client makes (block import, authoring, pool validation), so the
//!   `gpu_verify` host functions of cess-gpu-verify-runtime find it.
//! * `run` watches the transaction pool, asks the runtime which (TEE BLS
//!   signature, signed message, TEE key) records the new transactions will
//!   verify (runtime API `GpuVerifyRecords::verify_records`; the runtime owns
//!   the storage the records need) and verifies all of them in ONE GPU batch
//!   (GpuState::batch_codes -> cess_bls_cache_verify_var) ahead of block
//!   execution.  The verdicts land in the C library's bounded verdict cache,
//!   so the runtime's per-extrinsic `gpu_verify::verify_bls` host call is a
//!   lookup.  The cache only ever holds GPU verdicts (bit-exact with the
//!   reference crate), never "unavailable", so a cold cache or no batcher
//!   changes timing, never results.
use crate::primitives::Block;
use cess_gpu_verify_runtime::{
	ext::{GpuState, GpuVerifierExt},
	GpuVerifyRecords,
};
use futures::{FutureExt, StreamExt};
use sc_transaction_pool_api::{InPoolTransaction, TransactionPool};
use sp_api::ProvideRuntimeApi;
use sp_blockchain::HeaderBackend;
use sp_runtime::generic::BlockId;
use std::sync::Arc;

/// `ExtensionsFactory` of sc-client-api at polkadot-v0.9.36: one method,
/// called with the capabilities of the execution context.
pub struct GpuExtensionsFactory(pub Arc<GpuState>);

impl sc_client_api::execution_extensions::ExtensionsFactory for GpuExtensionsFactory {
	fn extensions_for(&self, _capabilities: sp_core::offchain::Capabilities) -> sp_externalities::Extensions {
		let mut e = sp_externalities::Extensions::new();
		e.register(GpuVerifierExt(self.0.clone()));
		e
	}
}

/// Records verified per GPU batch at most (one launch chunk of the library).
const MAX_BATCH: usize = 1 << 20;

/// The batcher task (spawned blocking: the GPU call blocks its thread).
pub async fn run<P, C>(pool: Arc<P>, client: Arc<C>, gpu: Arc<GpuState>)
where
	P: TransactionPool<Block = Block> + 'static,
	C: ProvideRuntimeApi<Block> + HeaderBackend<Block> + Send + Sync + 'static,
	C::Api: GpuVerifyRecords<Block>,
{
	let mut imported = pool.import_notification_stream();
	loop {
		// wait for one import, then take every notification already queued:
		// what arrived while the previous batch ran is verified as one batch
		let mut hashes = match imported.next().await {
			Some(h) => vec![h],
			None => return, // pool gone: node shutting down
		};
		while hashes.len() < MAX_BATCH {
			match imported.next().now_or_never() {
				Some(Some(h)) => hashes.push(h),
				Some(None) => return,
				None => break,
			}
		}
		let xts: Vec<_> =
			hashes.iter().filter_map(|h| pool.ready_transaction(h)).map(|tx| tx.data().clone()).collect();
		if xts.is_empty() {
			continue
		}
		// the runtime builds the records against the best block's state
		let best = client.info().best_hash;
		let records = match client.runtime_api().verify_records(&BlockId::Hash(best), xts) {
			Ok(r) if !r.is_empty() => r,
			_ => continue,
		};
		let recs: Vec<(&[u8], &[u8], &[u8])> = records.iter().map(|(s, m, k)| (&s[..], &m[..], &k[..])).collect();
		let _ = gpu.batch_codes(&recs);
	}
}
