/*
 * cess_bls.h — C ABI of the MI355X batch BLS12-381 verifier for CESS.
 *
 * Drop-in boundary for the reference crate `ic-verify-bls-signature`
 * (/root/reference/utils/verify-bls-signatures, Cargo.toml:2).  Each entry point
 * names the reference interface it replaces.  Plain pointers and sizes only; the
 * caller owns every buffer.  A context is used by one host thread at a time.
 *
 * Return values of every function are INFRASTRUCTURE status (CESS_BLS_OK or a
 * negative CESS_BLS_E_* code).  Verification verdicts are returned separately as
 * per-signature codes:
 *
 *   0 OK             verify_bls_signature(..) == Ok(())
 *   1 SIG_LEN        Signature::deserialize -> InvalidSignature::WrongLength  (src/lib.rs:139-142)
 *   2 SIG_POINT      Signature::deserialize -> InvalidSignature::InvalidPoint (src/lib.rs:147-149)
 *   3 PK_LEN         PublicKey::deserialize -> InvalidPublicKey::WrongLength  (src/lib.rs:69-72)
 *   4 PK_POINT       PublicKey::deserialize -> InvalidPublicKey::InvalidPoint (src/lib.rs:77-79)
 *   5 PAIRING_FAIL   PublicKey::verify -> Err(())                            (src/lib.rs:95-99)
 *
 * Precedence follows the reference (src/lib.rs:244-246): signature first, then
 * key, then the pairing.  Codes 1..5 all map to the reference's Err(()).
 * Verdict bitmap: bit (i % 64) of word i / 64, LSB first, is 1 iff code i == 0.
 */
#ifndef CESS_BLS_H
#define CESS_BLS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CESS_BLS_OK 0
#define CESS_BLS_E_INVALID_ARG (-1)
#define CESS_BLS_E_NO_DEVICE (-2)
#define CESS_BLS_E_HIP (-3)
#define CESS_BLS_E_OOM (-4)
#define CESS_BLS_E_RCCL (-5)

enum cess_bls_code {
  CESS_BLS_CODE_OK = 0,
  CESS_BLS_CODE_SIG_LEN = 1,
  CESS_BLS_CODE_SIG_POINT = 2,
  CESS_BLS_CODE_PK_LEN = 3,
  CESS_BLS_CODE_PK_POINT = 4,
  CESS_BLS_CODE_PAIRING_FAIL = 5
};

#define CESS_BLS_SIG_BYTES 48  /* Signature::BYTES  src/lib.rs:126 */
#define CESS_BLS_PK_BYTES 96   /* PublicKey::BYTES  src/lib.rs:56  */
#define CESS_BLS_SK_BYTES 32   /* PrivateKey::BYTES src/lib.rs:178 */
#define CESS_BLS_GT_BYTES 576

typedef struct cess_bls_ctx cess_bls_ctx;

typedef struct cess_bls_config {
  int device;          /* HIP device ordinal (-1: current device)                  */
  uint64_t max_batch;  /* signatures per device launch chunk (0: default 1<<20)    */
  uint32_t flags;      /* CESS_BLS_F_* */
} cess_bls_config;

#define CESS_BLS_F_PROFILE 1u /* record per-stage HIP event timings */

/* Context: device buffers, stream, and the G2PREPARED_NEG_G table
 * (replaces the lazy_static at src/lib.rs:19-21). */
int cess_bls_ctx_create(const cess_bls_config* cfg, cess_bls_ctx** out);
void cess_bls_ctx_destroy(cess_bls_ctx* ctx);

/* verify_bls_signature(sig, msg, key) -> Result<(), ()>   (src/lib.rs:243-247)
 * Any lengths are accepted; *code_out receives the verdict code. */
int cess_bls_verify(cess_bls_ctx* ctx, const uint8_t* sig, size_t sig_len, const uint8_t* msg,
                    size_t msg_len, const uint8_t* key, size_t key_len, uint8_t* code_out);

/* verify_batch (new), fixed-stride fast path: n records of
 * 48-byte signatures and 96-byte keys; message i is msgs[msg_offsets[i] ..
 * msg_offsets[i+1]).  codes_out: n bytes (may be NULL); bitmap_out:
 * ceil(n/64) words (may be NULL).  Host buffers. */
int cess_bls_verify_batch(cess_bls_ctx* ctx, size_t n, const uint8_t* sigs, const uint8_t* pks,
                          const uint8_t* msgs, const uint64_t* msg_offsets, uint8_t* codes_out,
                          uint64_t* bitmap_out);

/* verify_batch for arbitrary-length encodings (reference accepts any &[u8]):
 * record i is sig_data[sig_offsets[i]..sig_offsets[i+1]) etc.  Host buffers. */
int cess_bls_verify_batch_var(cess_bls_ctx* ctx, size_t n, const uint8_t* sig_data,
                              const uint64_t* sig_offsets, const uint8_t* pk_data, const uint64_t* pk_offsets,
                              const uint8_t* msgs, const uint64_t* msg_offsets, uint8_t* codes_out,
                              uint64_t* bitmap_out);

/* Device-resident fixed-stride batch: all pointers are device (HBM) pointers;
 * work is enqueued on `stream` (a hipStream_t; NULL = the context's stream) and
 * NOT synchronised.  bitmap words are written for whole 64-signature groups;
 * n must be a multiple of 64 unless it is the whole batch. */
int cess_bls_verify_batch_device(cess_bls_ctx* ctx, size_t n, const uint8_t* d_sigs, const uint8_t* d_pks,
                                 const uint8_t* d_msgs, const uint64_t* d_msg_offsets, uint8_t* d_codes,
                                 uint64_t* d_bitmap, void* stream);

/* Distinct-key table (key decode and G2Prepared are
 * "cacheable per distinct pk"; §8(f) rank 3).  Decodes k 96-byte keys
 * (PublicKey::deserialize, src/lib.rs:68-82) and prepares their line
 * coefficients (G2Prepared::from, src/lib.rs:88) once, on the device;
 * key_codes_out (k bytes, may be NULL) receives 0 or CESS_BLS_PK_POINT.
 * Replaces the context's previous table.  Host buffer. */
int cess_bls_keys_load(cess_bls_ctx* ctx, size_t k, const uint8_t* pks, uint8_t* key_codes_out);

/* Keyed batch: signature i (48 B) over message i is verified against loaded
 * key key_idx[i] (< k, checked; else CESS_BLS_E_INVALID_ARG).  Codes and
 * bitmap equal cess_bls_verify_batch on the expanded records (same
 * precedence: signature first, src/lib.rs:244-245).  Host buffers. */
int cess_bls_verify_batch_keyed(cess_bls_ctx* ctx, size_t n, const uint8_t* sigs, const uint32_t* key_idx,
                                const uint8_t* msgs, const uint64_t* msg_offsets, uint8_t* codes_out,
                                uint64_t* bitmap_out);

/* Device-resident keyed batch (as cess_bls_verify_batch_device; the caller
 * guarantees every d_key_idx[i] < k). */
int cess_bls_verify_batch_keyed_device(cess_bls_ctx* ctx, size_t n, const uint8_t* d_sigs,
                                       const uint32_t* d_key_idx, const uint8_t* d_msgs,
                                       const uint64_t* d_msg_offsets, uint8_t* d_codes, uint64_t* d_bitmap,
                                       void* stream);

/* PrivateKey::public_key (src/lib.rs:226-228) for n 32-byte big-endian secret
 * keys (each must be < r, as PrivateKey::deserialize enforces at :208-223);
 * pks_out: n * 96 bytes. */
int cess_bls_public_key_batch(cess_bls_ctx* ctx, size_t n, const uint8_t* sks, uint8_t* pks_out);

/* PrivateKey::sign (src/lib.rs:233-236): sigs_out[i] = compress(sk_i * H(msg_i)). */
int cess_bls_sign_batch(cess_bls_ctx* ctx, size_t n, const uint8_t* sks, const uint8_t* msgs,
                        const uint64_t* msg_offsets, uint8_t* sigs_out);

/* hash_to_g1 (src/lib.rs:25-31), compressed 48-byte output; exposed for tests. */
int cess_bls_hash_to_g1_batch(cess_bls_ctx* ctx, size_t n, const uint8_t* msgs, const uint64_t* msg_offsets,
                              uint8_t* out48);

/* Gt value of PublicKey::verify's pairing product (576 bytes, 12 big-endian Fp
 * in tower order c0.c0.c0 .. c1.c2.c1) for valid (sig, pk) records; records
 * whose code != 0 get zeros.  Exposed so tests can pin Gt intermediates. */
int cess_bls_gt_batch(cess_bls_ctx* ctx, size_t n, const uint8_t* sigs, const uint8_t* pks, const uint8_t* msgs,
                      const uint64_t* msg_offsets, uint8_t* codes_out, uint8_t* gt_out);

/* ---- RLC batch mode (north_star "optional random-linear-combination batch
 * mode"; no reference counterpart).  For records with distinct keys
 * pk_1..pk_K, one check
 *     e(sum r_i sig_i, -G2) * prod_k e(sum_{pk_i = pk_k} r_i H(m_i), pk_k) == 1
 * (r_i: 128-bit, derived from `seed32` by SHA-256) replaces n pairing
 * products; a failing batch is bisected down to leaves verified per signature,
 * so codes_out equals cess_bls_verify_batch's except with probability 2^-127
 * per check.  Fixed-stride records (48-B sigs, 96-B keys), host buffers. */
int cess_bls_verify_batch_rlc(cess_bls_ctx* ctx, size_t n, const uint8_t* sigs, const uint8_t* pks,
                              const uint8_t* msgs, const uint64_t* msg_offsets, const uint8_t* seed32,
                              uint8_t* codes_out, uint64_t* bitmap_out,
                              uint64_t* stats4 /* checks, leaves, leaf sigs, distinct keys; may be NULL */);

/* Multi-GPU form (one shard per context): rlc_begin runs the shard's check and
 * returns its Gt partial (576 canonical bytes); the caller all-gathers the
 * partials (RCCL), combines them with cess_bls_gt_product_is_one, and passes
 * the global verdict to rlc_finish, which bisects the shard if needed.  The
 * record buffers must stay valid until rlc_finish returns. */
int cess_bls_rlc_begin(cess_bls_ctx* ctx, size_t n, const uint8_t* sigs, const uint8_t* pks, const uint8_t* msgs,
                       const uint64_t* msg_offsets, const uint8_t* seed32, uint8_t* gt_out);
int cess_bls_gt_product_is_one(cess_bls_ctx* ctx, size_t m, const uint8_t* gts, int* is_one);
int cess_bls_rlc_finish(cess_bls_ctx* ctx, int global_ok, uint8_t* codes_out, uint64_t* bitmap_out,
                        uint64_t* stats4);

/* Per-stage timings (ms, summed since the last reset) when CESS_BLS_F_PROFILE is
 * set.  names/ms arrays of length max; returns the number of stages. */
int cess_bls_stage_times(cess_bls_ctx* ctx, const char** names, double* ms, int max, int reset);

const char* cess_bls_status_string(int status);
const char* cess_bls_version(void);

#ifdef __cplusplus
}
#endif
#endif /* CESS_BLS_H */
