// UNCOMPILED SKETCH (no cargo here): the node-side batcher of SURVEY.md §8(f)
// rank 2.  It watches the transaction pool for `audit::submit_verify_result`
// extrinsics (patches/audit.rs), extracts each (tee BLS signature, signed
// message, TEE key) record and verifies all of them in ONE GPU batch
// (cess_bls_verify_batch_var) ahead of block execution.  The verdicts land in
// the GpuState cache, so the runtime's per-extrinsic `gpu_verify::verify_bls`
// host call is a hash lookup.  The cache only ever holds verdicts equal to the
// reference crate's, so a cold cache (or no batcher) changes timing, never
// results.
use cess_gpu_verify_runtime::ext::{batch_codes, GpuState};
use futures::StreamExt;
use std::sync::Arc;

const BATCH_WINDOW: std::time::Duration = std::time::Duration::from_millis(50);

pub async fn run<P>(pool: Arc<P>, gpu: Arc<GpuState>)
where
    P: sc_transaction_pool_api::TransactionPool<Block = node_primitives::Block> + 'static,
{
    let mut imported = pool.import_notification_stream();
    loop {
        // collect what arrived within the window, then verify it as one batch
        let mut hashes = Vec::new();
        if let Some(h) = imported.next().await {
            hashes.push(h);
        }
        let deadline = futures_timer::Delay::new(BATCH_WINDOW);
        futures::pin_mut!(deadline);
        loop {
            futures::select! {
                h = imported.next() => match h { Some(h) => hashes.push(h), None => break },
                _ = deadline.as_mut().fuse() => break,
            }
        }
        let (mut sigs, mut msgs, mut keys) = (Vec::new(), Vec::new(), Vec::new());
        for h in hashes {
            if let Some(tx) = pool.ready_transaction(&h) {
                // decode_verify_record: SCALE-decode the extrinsic; for
                // Audit::submit_verify_result return (tee_signature,
                // verify_result_message(..), TeeBlsKey of the signer) --
                // the same bytes the pallet passes to gpu_verify::verify_bls
                if let Some((s, m, k)) = crate::gpu_records::decode_verify_record(tx.data()) {
                    sigs.push(s);
                    msgs.push(m);
                    keys.push(k);
                }
            }
        }
        if !sigs.is_empty() {
            let gpu = gpu.clone();
            // one C-ABI batch call off the async executor
            let _ = tokio::task::spawn_blocking(move || batch_codes(&gpu, &sigs, &msgs, &keys)).await;
        }
    }
}
