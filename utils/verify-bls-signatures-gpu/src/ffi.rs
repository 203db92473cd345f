//! Raw bindings of include/cess_bls.h (one `extern "C"` item per header entry
//! point; the comments name the reference interface each one replaces).
//! NOT COMPILED in this repository's image (no cargo).
#![allow(non_camel_case_types)]

use core::ffi::{c_char, c_int, c_void};

pub const CESS_BLS_OK: c_int = 0;
pub const CESS_BLS_E_INVALID_ARG: c_int = -1;
pub const CESS_BLS_E_NO_DEVICE: c_int = -2;
pub const CESS_BLS_E_HIP: c_int = -3;
pub const CESS_BLS_E_OOM: c_int = -4;
pub const CESS_BLS_E_RCCL: c_int = -5;
pub const CESS_BLS_E_BUSY: c_int = -6;
pub const CESS_BLS_E_BAD_KEY: c_int = -7;
pub const CESS_BLS_E_BAD_SIG: c_int = -8;
pub const CESS_BLS_E_NO_COMM: c_int = -9;
pub const CESS_BLS_E_COMM: c_int = -11;

pub const CODE_OK: u8 = 0;
pub const CODE_SIG_LEN: u8 = 1;
pub const CODE_SIG_POINT: u8 = 2;
pub const CODE_PK_LEN: u8 = 3;
pub const CODE_PK_POINT: u8 = 4;
pub const CODE_PAIRING_FAIL: u8 = 5;
/// no verdict (cache path without a device / failed batch): the caller decides
pub const CODE_UNAVAILABLE: u8 = 0xff;
pub const CESS_BLS_KIND_SIG: c_int = 0;
pub const CESS_BLS_KIND_PK: c_int = 1;
pub const CESS_BLS_COMM_NAME_BYTES: usize = 64;

pub const CESS_BLS_F_PROFILE: u32 = 1;
pub const CESS_BLS_F_STRICT_IDENTITY: u32 = 2;
pub const CESS_BLS_F_RLC_DISTINCT: u32 = 4;
pub const CESS_BLS_MODE_PER_SIG: u32 = 0;
pub const CESS_BLS_MODE_RLC: u32 = 1;
pub const CESS_BLS_COMM_ID_BYTES: usize = 128;
pub const CESS_BLS_BUS_ID_BYTES: usize = 32;

#[repr(C)]
pub struct cess_bls_config {
    pub device: c_int,
    pub max_batch: u64,
    pub flags: u32,
    pub mode: u32,
    pub n_devices: c_int,
    pub devices: *const c_int,
}

#[repr(C)]
pub struct cess_bls_ctx {
    _private: [u8; 0],
}
#[repr(C)]
pub struct cess_bls_comm {
    _private: [u8; 0],
}
#[repr(C)]
pub struct cess_bls_cache {
    _private: [u8; 0],
}

extern "C" {
    // context (G2PREPARED_NEG_G, utils/verify-bls-signatures/src/lib.rs:19-21, plus device state)
    pub fn cess_bls_ctx_create(cfg: *const cess_bls_config, out: *mut *mut cess_bls_ctx) -> c_int;
    pub fn cess_bls_ctx_destroy(ctx: *mut cess_bls_ctx);
    // verify_bls_signature (src/lib.rs:243-247)
    pub fn cess_bls_verify(ctx: *mut cess_bls_ctx, sig: *const u8, sig_len: usize, msg: *const u8, msg_len: usize,
                           key: *const u8, key_len: usize, code_out: *mut u8) -> c_int;
    // verify_batch (new)
    pub fn cess_bls_verify_batch(ctx: *mut cess_bls_ctx, n: usize, sigs: *const u8, pks: *const u8, msgs: *const u8,
                                 msg_offsets: *const u64, codes_out: *mut u8, bitmap_out: *mut u64) -> c_int;
    pub fn cess_bls_verify_batch_var(ctx: *mut cess_bls_ctx, n: usize, sig_data: *const u8, sig_offsets: *const u64,
                                     pk_data: *const u8, pk_offsets: *const u64, msgs: *const u8,
                                     msg_offsets: *const u64, codes_out: *mut u8, bitmap_out: *mut u64) -> c_int;
    pub fn cess_bls_verify_batch_device(ctx: *mut cess_bls_ctx, n: usize, d_sigs: *const u8, d_pks: *const u8,
                                        d_msgs: *const u8, d_msg_offsets: *const u64, d_codes: *mut u8,
                                        d_bitmap: *mut u64, stream: *mut c_void) -> c_int;
    // distinct-key table (PublicKey::deserialize :68-82 + G2Prepared::from :88 once per key)
    pub fn cess_bls_keys_load(ctx: *mut cess_bls_ctx, k: usize, pks: *const u8, key_codes_out: *mut u8) -> c_int;
    pub fn cess_bls_verify_batch_keyed(ctx: *mut cess_bls_ctx, n: usize, sigs: *const u8, key_idx: *const u32,
                                       msgs: *const u8, msg_offsets: *const u64, codes_out: *mut u8,
                                       bitmap_out: *mut u64) -> c_int;
    pub fn cess_bls_verify_batch_keyed_device(ctx: *mut cess_bls_ctx, n: usize, d_sigs: *const u8,
                                              d_key_idx: *const u32, d_msgs: *const u8, d_msg_offsets: *const u64,
                                              d_codes: *mut u8, d_bitmap: *mut u64, stream: *mut c_void) -> c_int;
    // PrivateKey::public_key (:226-228), PrivateKey::sign (:233-236), hash_to_g1 (:25-31)
    pub fn cess_bls_public_key_batch(ctx: *mut cess_bls_ctx, n: usize, sks: *const u8, pks_out: *mut u8) -> c_int;
    pub fn cess_bls_sign_batch(ctx: *mut cess_bls_ctx, n: usize, sks: *const u8, msgs: *const u8,
                               msg_offsets: *const u64, sigs_out: *mut u8) -> c_int;
    pub fn cess_bls_sign_batch_device(ctx: *mut cess_bls_ctx, n: usize, d_sks: *const u8, d_msgs: *const u8,
                                      d_msg_offsets: *const u64, d_sigs_out: *mut u8, stream: *mut c_void) -> c_int;
    pub fn cess_bls_hash_to_g1_batch(ctx: *mut cess_bls_ctx, n: usize, msgs: *const u8, msg_offsets: *const u64,
                                     out48: *mut u8) -> c_int;
    pub fn cess_bls_gt_batch(ctx: *mut cess_bls_ctx, n: usize, sigs: *const u8, pks: *const u8, msgs: *const u8,
                             msg_offsets: *const u64, codes_out: *mut u8, gt_out: *mut u8) -> c_int;
    // RLC batch mode (north_star); seed32 NULL = library CSPRNG
    pub fn cess_bls_verify_batch_rlc(ctx: *mut cess_bls_ctx, n: usize, sigs: *const u8, pks: *const u8,
                                     msgs: *const u8, msg_offsets: *const u64, seed32: *const u8,
                                     codes_out: *mut u8, bitmap_out: *mut u64, stats4: *mut u64) -> c_int;
    pub fn cess_bls_rlc_begin(ctx: *mut cess_bls_ctx, n: usize, sigs: *const u8, pks: *const u8, msgs: *const u8,
                              msg_offsets: *const u64, seed32: *const u8, gt_out: *mut u8) -> c_int;
    pub fn cess_bls_gt_product_is_one(ctx: *mut cess_bls_ctx, m: usize, gts: *const u8, is_one: *mut c_int) -> c_int;
    pub fn cess_bls_rlc_finish(ctx: *mut cess_bls_ctx, global_ok: c_int, codes_out: *mut u8, bitmap_out: *mut u64,
                               stats4: *mut u64) -> c_int;
    // multi-GPU: RCCL communicator in the context
    pub fn cess_bls_comm_id(id_out: *mut u8) -> c_int;
    pub fn cess_bls_comm_init(ctx: *mut cess_bls_ctx, nranks: c_int, rank: c_int, id: *const u8) -> c_int;
    pub fn cess_bls_shard_range(n: u64, nranks: c_int, rank: c_int, begin: *mut u64, end: *mut u64,
                                words_per_rank: *mut u64) -> c_int;
    pub fn cess_bls_verify_batch_sharded(ctx: *mut cess_bls_ctx, n: usize, sigs: *const u8, pks: *const u8,
                                         msgs: *const u8, msg_offsets: *const u64, codes_out: *mut u8,
                                         bitmap_out: *mut u64) -> c_int;
    /// Collective and BLOCKING: returns after the final status agreement, which
    /// waits for the verdict all-gathers on the host (include/cess_bls.h).
    pub fn cess_bls_verify_batch_sharded_device(ctx: *mut cess_bls_ctx, n_total: usize, d_sigs: *const u8,
                                                d_pks: *const u8, d_msgs: *const u8, d_msg_offsets: *const u64,
                                                d_codes_all: *mut u8, d_bitmap_all: *mut u64,
                                                stream: *mut c_void) -> c_int;
    pub fn cess_bls_verify_batch_rlc_sharded(ctx: *mut cess_bls_ctx, n_shard: usize, sigs: *const u8,
                                             pks: *const u8, msgs: *const u8, msg_offsets: *const u64,
                                             seed32: *const u8, codes_out: *mut u8, bitmap_out: *mut u64,
                                             stats4: *mut u64, global_ok_out: *mut c_int) -> c_int;
    pub fn cess_bls_comm_barrier(ctx: *mut cess_bls_ctx) -> c_int;
    pub fn cess_bls_comm_max_f64(ctx: *mut cess_bls_ctx, value: *mut f64) -> c_int;
    pub fn cess_bls_comm_kind(ctx: *mut cess_bls_ctx) -> *const c_char;
    pub fn cess_bls_comm_info(ctx: *mut cess_bls_ctx, nranks_out: *mut c_int, rank_out: *mut c_int,
                              bus_ids_out: *mut c_char) -> c_int;
    pub fn cess_bls_verify_batch_var_sharded(ctx: *mut cess_bls_ctx, n: usize, sig_data: *const u8,
                                             sig_offsets: *const u64, pk_data: *const u8, pk_offsets: *const u64,
                                             msgs: *const u8, msg_offsets: *const u64, codes_out: *mut u8,
                                             bitmap_out: *mut u64) -> c_int;
    // host shared-memory transport of the sharded entry points (ranks on one host)
    pub fn cess_bls_comm_shm_name(name_out: *mut c_char) -> c_int;
    pub fn cess_bls_comm_init_shm(ctx: *mut cess_bls_ctx, nranks: c_int, rank: c_int, name: *const c_char) -> c_int;
    pub fn cess_bls_comm_open_shm(name: *const c_char, nranks: c_int, rank: c_int,
                                  out: *mut *mut cess_bls_comm) -> c_int;
    pub fn cess_bls_comm_close(comm: *mut cess_bls_comm);
    pub fn cess_bls_comm_agree(comm: *mut cess_bls_comm, status: c_int, agreed_out: *mut c_int) -> c_int;
    pub fn cess_bls_comm_gather_verdicts(comm: *mut cess_bls_comm, n_total: u64, shard_codes: *const u8,
                                         codes_out: *mut u8, bitmap_out: *mut u64) -> c_int;
    // Signature::deserialize (:138-152) / PublicKey::deserialize (:68-82) alone
    pub fn cess_bls_deserialize_batch(ctx: *mut cess_bls_ctx, kind: c_int, n: usize, data: *const u8,
                                      offsets: *const u64, codes_out: *mut u8) -> c_int;
    // bounded verdict cache (node host function + batcher)
    pub fn cess_bls_cache_create(capacity: usize, out: *mut *mut cess_bls_cache) -> c_int;
    pub fn cess_bls_cache_destroy(cache: *mut cess_bls_cache);
    pub fn cess_bls_cache_clear(cache: *mut cess_bls_cache) -> c_int;
    pub fn cess_bls_cache_size(cache: *mut cess_bls_cache) -> usize;
    pub fn cess_bls_cache_verify_var(cache: *mut cess_bls_cache, ctx: *mut cess_bls_ctx, n: usize,
                                     sig_data: *const u8, sig_offsets: *const u64, pk_data: *const u8,
                                     pk_offsets: *const u64, msgs: *const u8, msg_offsets: *const u64,
                                     codes_out: *mut u8, stats3: *mut u64) -> c_int;
    pub fn cess_bls_cache_insert_var(cache: *mut cess_bls_cache, n: usize, sig_data: *const u8,
                                     sig_offsets: *const u64, pk_data: *const u8, pk_offsets: *const u64,
                                     msgs: *const u8, msg_offsets: *const u64, codes: *const u8) -> c_int;
    pub fn cess_bls_sha256(data: *const u8, len: usize, out: *mut u8) -> c_int;
    // device memory on the context's GPU
    pub fn cess_bls_device_alloc(ctx: *mut cess_bls_ctx, bytes: usize, d_out: *mut *mut c_void) -> c_int;
    pub fn cess_bls_device_free(ctx: *mut cess_bls_ctx, d: *mut c_void) -> c_int;
    pub fn cess_bls_copy_to_device(ctx: *mut cess_bls_ctx, d_dst: *mut c_void, src: *const c_void,
                                   bytes: usize) -> c_int;
    pub fn cess_bls_copy_from_device(ctx: *mut cess_bls_ctx, dst: *mut c_void, d_src: *const c_void,
                                     bytes: usize) -> c_int;
    pub fn cess_bls_synchronize(ctx: *mut cess_bls_ctx) -> c_int;
    // cp_enclave_verify::verify_bls (primitives/enclave-verify/src/lib.rs:230-235)
    pub fn cess_bls_enclave_verify_bls(ctx: *mut cess_bls_ctx, key: *const u8, key_len: usize, msg: *const u8,
                                       msg_len: usize, sig: *const u8, sig_len: usize, ok_out: *mut c_int) -> c_int;
    // diagnostics
    pub fn cess_bls_stage_times(ctx: *mut cess_bls_ctx, names: *mut *const c_char, ms: *mut f64, max: c_int,
                                reset: c_int) -> c_int;
    pub fn cess_bls_stage_stats(ctx: *mut cess_bls_ctx, names: *mut *const c_char, ms: *mut f64, launches: *mut u64,
                                max: c_int, reset: c_int) -> c_int;
    pub fn cess_bls_launch_records(ctx: *mut cess_bls_ctx) -> u64;
    pub fn cess_bls_status_string(status: c_int) -> *const c_char;
    pub fn cess_bls_version() -> *const c_char;
    pub fn cess_bls_device_count() -> c_int;

    // include/cess_rsa.h: cp_enclave_verify::verify_rsa (primitives/enclave-verify/src/lib.rs:221-228)
    pub fn cess_rsa_parse_key(der: *const u8, len: usize, format: c_int, n_out: *mut u8, n_cap: usize,
                              n_len: *mut usize, e_out: *mut u64) -> c_int;
    pub fn cess_rsa_keys_load(ctx: *mut cess_bls_ctx, k: usize, ders: *const u8, der_offsets: *const u64,
                              format: c_int, key_status_out: *mut c_int) -> c_int;
    pub fn cess_rsa_verify_batch(ctx: *mut cess_bls_ctx, n: usize, key_idx: *const u32, sigs: *const u8,
                                 sig_offsets: *const u64, msgs: *const u8, msg_offsets: *const u64,
                                 codes_out: *mut u8, bitmap_out: *mut u64) -> c_int;
    pub fn cess_rsa_verify(ctx: *mut cess_bls_ctx, key_der: *const u8, key_len: usize, msg: *const u8,
                           msg_len: usize, sig: *const u8, sig_len: usize, ok_out: *mut c_int) -> c_int;
    pub fn cess_rsa_verify_batch_device(ctx: *mut cess_bls_ctx, n: usize, d_key_idx: *const u32, d_sigs: *const u8,
                                        d_sig_offsets: *const u64, d_msgs: *const u8, d_msg_offsets: *const u64,
                                        d_codes: *mut u8, stream: *mut c_void) -> c_int;
}

pub const CESS_RSA_E_UNSUPPORTED: c_int = -10;
pub const CESS_RSA_KEY_SPKI: c_int = 0;
pub const CESS_RSA_KEY_PKCS1: c_int = 1;
pub const RSA_CODE_OK: u8 = 0;
