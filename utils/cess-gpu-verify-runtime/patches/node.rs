// UNCOMPILED (no cargo here) -- what node/src adds to route the gpu_verify
// host functions (../src/lib.rs) to an MI355X.  Replaces nothing: the
// reference executor exposes only the benchmarking host functions
// (node/src/executor.rs:8).  The batcher task is patches/node_batcher.rs
// (node/src/gpu_batcher.rs).

// --- node/src/executor.rs ---------------------------------------------------
impl sc_executor::NativeExecutionDispatch for ExecutorDispatch {
    // the runtime may now import `gpu_verify::*` host functions
    type ExtendHostFunctions = (
        frame_benchmarking::benchmarking::HostFunctions,
        cess_gpu_verify_runtime::gpu_verify::HostFunctions,
    );
    // dispatch / native_version unchanged
}

// --- node/src/service.rs ------------------------------------------------------
// One GPU context per node process; the extension is attached to every
// runtime call that executes blocks or validates transactions, so block import,
// block authoring and the transaction pool all see the same verdict cache.
pub struct GpuExtensionsFactory(pub std::sync::Arc<cess_gpu_verify_runtime::ext::GpuState>);

impl sc_client_api::execution_extensions::ExtensionsFactory<Block> for GpuExtensionsFactory {
    fn extensions_for(
        &self,
        _block_hash: <Block as sp_runtime::traits::Block>::Hash,
        _block_number: sp_runtime::traits::NumberFor<Block>,
    ) -> sp_externalities::Extensions {
        let mut e = sp_externalities::Extensions::new();
        e.register(cess_gpu_verify_runtime::ext::GpuVerifierExt(self.0.clone()));
        e
    }
}

// in new_partial(), after the client is built (no GPU: GpuState still comes
// up, every host call answers UNAVAILABLE and the runtime's wasm path runs):
//     if let Some(gpu) = cess_gpu_verify_runtime::ext::GpuState::new(&verify_bls_signatures_gpu::Config {
//         device: config.gpu_device.unwrap_or(0), max_batch: 1 << 20, ..Default::default() }) {
//         client.execution_extensions().set_extensions_factory(GpuExtensionsFactory(gpu.clone()));
//         task_manager.spawn_handle().spawn("gpu-verify-batcher", None,
//             crate::gpu_batcher::run(transaction_pool.clone(), client.clone(), gpu));
//     }
