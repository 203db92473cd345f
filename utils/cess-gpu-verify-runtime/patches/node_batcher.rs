// UNCOMPILED (no cargo here) -- node/src/gpu_batcher.rs: the node-side batcher
// of SURVEY.md §8(f) rank 2.  It watches the transaction pool, asks the
// runtime which (TEE BLS signature, signed message, TEE key) records the new
// transactions will verify (runtime API `GpuVerifyRecords::verify_records`,
// implemented with `decode_verify_record` in patches/audit.rs -- the runtime
// owns the storage the records need), and verifies all of them in ONE GPU
// batch (GpuState::batch_codes -> cess_bls_cache_verify_var) ahead of block
// execution.  The verdicts land in the C library's bounded verdict cache, so
// the runtime's per-extrinsic `gpu_verify::verify_bls` host call is a lookup.
// The cache only ever holds GPU verdicts (bit-exact with the reference crate),
// never "unavailable", so a cold cache or no batcher changes timing, never
// results.
use cess_gpu_verify_runtime::{ext::GpuState, GpuVerifyRecords};
use futures::{FutureExt, StreamExt};
use sc_transaction_pool_api::{InPoolTransaction, TransactionPool};
use sp_api::ProvideRuntimeApi;
use sp_blockchain::HeaderBackend;
use std::sync::Arc;

/// Transactions collected per batch: within this window after the first
/// import notification (a GPU batch of a few thousand records costs about as
/// much as one record, DESIGN.md §1 latency).
const BATCH_WINDOW: std::time::Duration = std::time::Duration::from_millis(50);

pub async fn run<P, C>(pool: Arc<P>, client: Arc<C>, gpu: Arc<GpuState>)
where
    P: TransactionPool<Block = node_primitives::Block> + 'static,
    C: ProvideRuntimeApi<node_primitives::Block> + HeaderBackend<node_primitives::Block> + Send + Sync + 'static,
    C::Api: GpuVerifyRecords<node_primitives::Block>,
{
    let mut imported = pool.import_notification_stream();
    loop {
        // collect what arrives within the window, then verify it as one batch
        let mut hashes = Vec::new();
        match imported.next().await {
            Some(h) => hashes.push(h),
            None => return,   // pool gone: node shutting down
        }
        let deadline = futures_timer::Delay::new(BATCH_WINDOW).fuse();
        futures::pin_mut!(deadline);
        loop {
            futures::select! {
                h = imported.next().fuse() => match h { Some(h) => hashes.push(h), None => break },
                _ = deadline => break,
            }
        }
        let xts: Vec<_> = hashes.iter().filter_map(|h| pool.ready_transaction(h)).map(|tx| tx.data().clone()).collect();
        if xts.is_empty() {
            continue;
        }
        // the runtime builds the records against the best block's state
        let best = client.info().best_hash;
        let records = match client.runtime_api().verify_records(best, xts) {
            Ok(r) if !r.is_empty() => r,
            _ => continue,
        };
        let gpu = gpu.clone();
        // one C-ABI batch call off the async executor; the codes are cached
        let _ = tokio::task::spawn_blocking(move || {
            let recs: Vec<(&[u8], &[u8], &[u8])> =
                records.iter().map(|(s, m, k)| (&s[..], &m[..], &k[..])).collect();
            gpu.batch_codes(&recs)
        })
        .await;
    }
}
