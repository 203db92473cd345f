/*
 * cess_bls.h — C ABI of the MI355X batch BLS12-381 verifier for CESS.
 *
 * Drop-in boundary for the reference crate `ic-verify-bls-signature`
 * (/root/reference/utils/verify-bls-signatures, Cargo.toml:2).  Each entry point
 * names the reference interface it replaces.  Plain pointers and sizes only; the
 * caller owns every buffer.  A context is used by one host thread at a time.
 *
 * Concurrency: a context is used by one host thread at a time; a call that
 * finds another thread inside the same context returns CESS_BLS_E_BUSY.
 * Successive calls on one context are ordered on the device even when they
 * name different streams (each call waits for the previous call's work).
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
#define CESS_BLS_E_BUSY (-6)     /* another host thread is inside a call on this context */
#define CESS_BLS_E_BAD_KEY (-7)  /* cess_bls_enclave_verify_bls: the key does not deserialize (the reference panics) */
#define CESS_BLS_E_BAD_SIG (-8)  /* cess_bls_enclave_verify_bls: the signature does not deserialize (the reference panics) */
#define CESS_BLS_E_NO_COMM (-9)  /* a sharded entry point on a context without cess_bls_comm_init[_shm] */
/* (-10 is CESS_RSA_E_UNSUPPORTED, include/cess_rsa.h) */
#define CESS_BLS_E_COMM (-11)    /* communicator (RCCL or shm): a peer timed out (CESS_BLS_COMM_TIMEOUT_MS) or the
                                    communicator was aborted; every later collective on it fails the same way */

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
#define CESS_BLS_COMM_ID_BYTES 128  /* ncclUniqueId */
#define CESS_BLS_COMM_NAME_BYTES 64  /* cess_bls_comm_shm_name */
#define CESS_BLS_BUS_ID_BYTES 32     /* cess_bls_comm_info: one NUL-padded PCI bus id per rank */

typedef struct cess_bls_ctx cess_bls_ctx;

/* Context configuration (SURVEY §8(b) bls_ctx_create: device set, batch size,
 * mode, strict-identity flag).  Zero-initialise and set what you need. */
typedef struct cess_bls_config {
  int device;          /* HIP device ordinal of a single-device context (-1: device 0)           */
  uint64_t max_batch;  /* signatures per device launch chunk (0: default 1<<20)                  */
  uint32_t flags;      /* CESS_BLS_F_*                                                            */
  uint32_t mode;       /* CESS_BLS_MODE_*: what cess_bls_verify_batch runs                       */
  int n_devices;       /* > 1: one context over several GPUs of this process: host-buffer batches
                          are sharded by index across them (one host thread per device)          */
  const int* devices;  /* n_devices ordinals (NULL: 0 .. n_devices-1); may repeat an ordinal      */
} cess_bls_config;

#define CESS_BLS_F_PROFILE 1u          /* record per-stage HIP event timings */
/* Reject identity public keys (0xc0 || 0^95) with CESS_BLS_CODE_PK_POINT, as the
 * IETF KeyValidate does.  Off by default: the reference accepts them
 * (PublicKey::deserialize, src/lib.rs:68-82, has no identity check), so the
 * (sig = O, pk = O) pair verifies for every message. */
#define CESS_BLS_F_STRICT_IDENTITY 2u
/* RLC mode for batches of (mostly) distinct keys: no key grouping; every record
 * keeps its own Miller value Miller(r_i H(m_i), pk_i) -- one pairing per record
 * instead of two -- the check multiplies them with Miller(sum r_i sig_i, -G2)
 * under ONE final exponentiation, and bisection reuses the stored values (a
 * level costs one S sum, one Miller loop and one final exponentiation per
 * range).  Codes are those of cess_bls_verify_batch (leaves of 2,048 records
 * are verified per signature).  Its random exponents take 2^63 values
 * (a + b lambda with 32-bit a, b and lambda the G1 endomorphism's eigenvalue:
 * a check passes an invalid batch with probability <= 2^-63; Ethereum
 * consensus clients batch BLS with 64-bit exponents); the key-grouped mode's
 * are 128-bit. */
#define CESS_BLS_F_RLC_DISTINCT 4u

#define CESS_BLS_MODE_PER_SIG 0u  /* two-pairing check per signature (default; src/lib.rs:85-100)      */
/* random linear combination with bisection (cess_bls_verify_batch_rlc semantics):
 * cess_bls_verify_batch draws a fresh 32-byte seed from the OS CSPRNG per call */
#define CESS_BLS_MODE_RLC 1u

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

/* Device-resident keyed batch (as cess_bls_verify_batch_device).  A record whose
 * d_key_idx[i] >= k is rejected on the device with CESS_BLS_CODE_PK_POINT (its
 * key does not exist), so no out-of-range table row is ever read. */
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

/* cess_bls_sign_batch over device buffers (d_sks: n * 32 B, d_msgs with n + 1
 * offsets, d_sigs_out: n * 48 B), enqueued on `stream` (null: the context's)
 * without waiting: the batch signer of the TEE side. */
int cess_bls_sign_batch_device(cess_bls_ctx* ctx, size_t n, const uint8_t* d_sks, const uint8_t* d_msgs,
                               const uint64_t* d_msg_offsets, uint8_t* d_sigs_out, void* stream);

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
 * (r_i: 128-bit, r_i = SHA-256(seed32 || index)[0:16] | 1) replaces n pairing
 * products; a failing batch is bisected down to leaves verified per signature,
 * so codes_out equals cess_bls_verify_batch's except with probability 2^-127
 * per check.  Fixed-stride records (48-B sigs, 96-B keys), host buffers.
 *
 * SECURITY: seed32 MUST be secret and unpredictable to whoever produced the
 * signatures (fresh CSPRNG output per call, never reused, never derived from
 * the batch).  With a seed the signer can predict, forgeries can be crafted
 * whose errors cancel in the combination and the batch reports them valid.
 * Pass seed32 = NULL to have the library draw one from the OS CSPRNG
 * (getrandom(2)).  Batches with more than one distinct key per 8 records gain
 * nothing from a combination and are verified per signature.
 * The sums of a check are formed by 8-bit-window buckets (Pippenger) when the
 * check has at most 256 segments (one segment per range of records and per
 * key group met) and 64 records per segment, else from each record's
 * multiples; env CESS_BLS_RLC_MSM=0 forces the latter, =1 the buckets whenever
 * the tables fit (tests).  Both give the same group elements.  Memory bound of
 * the bucket pass: 4,096 buckets x ~180 B per segment on the device (<= 190 MB
 * at 256 segments, kept by the context for reuse) and three host vectors of
 * 4 B per bucket (<= 12 MB) per check. */
int cess_bls_verify_batch_rlc(cess_bls_ctx* ctx, size_t n, const uint8_t* sigs, const uint8_t* pks,
                              const uint8_t* msgs, const uint64_t* msg_offsets, const uint8_t* seed32,
                              uint8_t* codes_out, uint64_t* bitmap_out,
                              uint64_t* stats4 /* checks, leaves, leaf sigs, distinct keys; may be NULL */);

/* Multi-GPU form driven by the caller's own collectives (one shard per
 * context): rlc_begin runs the shard's check and returns its Gt partial (576
 * canonical bytes); the caller all-gathers the partials, combines them with
 * cess_bls_gt_product_is_one (a batch-level verdict), and calls rlc_finish,
 * which bisects the shard whenever the shard's OWN check failed -- whatever
 * the combined verdict, so other shards' partials can never cancel a local
 * failure.  global_ok is accepted for the record only.  The record buffers
 * must stay valid until rlc_finish returns.  seed32 as above (NULL: OS CSPRNG). */
int cess_bls_rlc_begin(cess_bls_ctx* ctx, size_t n, const uint8_t* sigs, const uint8_t* pks, const uint8_t* msgs,
                       const uint64_t* msg_offsets, const uint8_t* seed32, uint8_t* gt_out);
int cess_bls_gt_product_is_one(cess_bls_ctx* ctx, size_t m, const uint8_t* gts, int* is_one);
int cess_bls_rlc_finish(cess_bls_ctx* ctx, int global_ok, uint8_t* codes_out, uint64_t* bitmap_out,
                        uint64_t* stats4);

/* ---- multi-GPU: communicator in the context ----
 * One process and one context per GPU.  Signatures are independent
 * (src/lib.rs:243 is per signature), so a batch shards by index with no
 * exchange during compute; the only collectives are all-gathers of the
 * verdict-bitmap words, of the code bytes, and in RLC mode of the 576-byte Gt
 * partials, plus a status agreement.
 *
 * Transports: RCCL over xGMI (cess_bls_comm_init; production) or host shared
 * memory (cess_bls_comm_init_shm; processes of one host, which may share one
 * GPU -- RCCL refuses two ranks on one device -- used to run the shard/merge
 * code with several ranks on a one-GPU box).  The sharded entry points behave
 * identically over either.
 *
 * Collective contract: every rank calls the same sharded entry points in the
 * same order.  Each call first agrees on the batch size and, after its local
 * work, on a status: when any rank fails (bad arguments, HIP error, OOM), EVERY
 * rank returns that failure (the most negative status) and no verdict data
 * moves, so one rank's error never leaves the others blocked in a collective. */

/* ncclGetUniqueId on one rank (e.g. rank 0); the caller distributes the 128
 * bytes to every rank out of band. */
int cess_bls_comm_id(uint8_t id_out[CESS_BLS_COMM_ID_BYTES]);
/* RCCL communicator on the context's device (collective: every rank calls it).
 * Created non-blocking (ncclCommInitRankConfig, blocking = 0); this call and
 * every later wait on the communicator poll ncclCommGetAsyncError against a
 * deadline, env CESS_BLS_COMM_TIMEOUT_MS (default 300000): a peer that never
 * arrives (or stops answering) makes this rank abort the communicator
 * (ncclCommAbort) and return CESS_BLS_E_COMM instead of hanging.  RCCL's
 * bootstrap blocks its calling thread until every rank connects, so the init
 * runs on a helper thread; when THIS call times out that thread stays blocked
 * inside RCCL, and the process should end with _exit() (static destructors
 * may otherwise run under it). */
int cess_bls_comm_init(cess_bls_ctx* ctx, int nranks, int rank, const uint8_t id[CESS_BLS_COMM_ID_BYTES]);
/* Records [*begin, *end) of rank's shard of an n-record batch: ceil(n/64)
 * bitmap words split into nranks equal runs of *words_per_rank words (the last
 * shards may be short or empty), so shards are whole bitmap words and the
 * all-gather needs no re-packing.  Pure function (no context). */
int cess_bls_shard_range(uint64_t n, int nranks, int rank, uint64_t* begin, uint64_t* end,
                         uint64_t* words_per_rank);
/* Sharded host-buffer batch (collective): every rank passes the WHOLE batch;
 * rank r verifies its shard, then codes and bitmap words are all-gathered, so
 * every rank returns the verdicts of all n records.  codes_out (n bytes) and
 * bitmap_out (ceil(n/64) words) may be NULL. */
int cess_bls_verify_batch_sharded(cess_bls_ctx* ctx, size_t n, const uint8_t* sigs, const uint8_t* pks,
                                  const uint8_t* msgs, const uint64_t* msg_offsets, uint8_t* codes_out,
                                  uint64_t* bitmap_out);
/* Sharded batch of arbitrary-length encodings (collective; the layout of
 * cess_bls_verify_batch_var, every rank passes the WHOLE batch): what node
 * callers holding &[u8] slices pass -- a wrong-length signature or key gets
 * its SIG_LEN / PK_LEN code in the gathered verdicts. */
int cess_bls_verify_batch_var_sharded(cess_bls_ctx* ctx, size_t n, const uint8_t* sig_data,
                                      const uint64_t* sig_offsets, const uint8_t* pk_data,
                                      const uint64_t* pk_offsets, const uint8_t* msgs,
                                      const uint64_t* msg_offsets, uint8_t* codes_out, uint64_t* bitmap_out);
/* Device-resident sharded batch (collective): d_sigs/d_pks/d_msgs/d_msg_offsets
 * hold only this rank's shard (cess_bls_shard_range; offsets shard-local,
 * shard_n + 1 entries).  d_bitmap_all (nranks * words_per_rank words) receives
 * the full batch bitmap; d_codes_all (nranks * words_per_rank * 64 bytes, may
 * be NULL) the full code array (bytes past n unspecified).  The work is
 * enqueued on `stream` (NULL: the context's); the call returns after a final
 * status agreement that waits for the all-gathers, so a failure on any rank
 * (also one after the work was enqueued) is returned on EVERY rank, and the
 * failing rank's gathered codes are CESS_BLS_CODE_UNAVAILABLE (no verdict).
 * BLOCKING: the host thread waits for the all-gathers before returning (since
 * round 4; before, the call only enqueued).  A caller that overlapped host
 * work with this call, or pipelined several calls, must move the call to a
 * thread of its own. */
int cess_bls_verify_batch_sharded_device(cess_bls_ctx* ctx, size_t n_total, const uint8_t* d_sigs,
                                         const uint8_t* d_pks, const uint8_t* d_msgs,
                                         const uint64_t* d_msg_offsets, uint8_t* d_codes_all,
                                         uint64_t* d_bitmap_all, void* stream);
/* RLC over the communicator (collective): each rank passes its own shard
 * (n_shard fixed-stride records), checks it with one combination (scalars
 * distinct across ranks), the Gt partials are all-gathered over RCCL and
 * multiplied on the device (*global_ok_out: the whole batch passed, may be
 * NULL), and a rank bisects iff its own check failed.  Codes/bitmap cover
 * the shard.  seed32 as cess_bls_verify_batch_rlc (every rank may pass its
 * own; NULL: OS CSPRNG). */
int cess_bls_verify_batch_rlc_sharded(cess_bls_ctx* ctx, size_t n_shard, const uint8_t* sigs, const uint8_t* pks,
                                      const uint8_t* msgs, const uint64_t* msg_offsets, const uint8_t* seed32,
                                      uint8_t* codes_out, uint64_t* bitmap_out, uint64_t* stats4,
                                      int* global_ok_out);
/* Control-plane helpers over the same communicator (collective). */
int cess_bls_comm_barrier(cess_bls_ctx* ctx);
int cess_bls_comm_max_f64(cess_bls_ctx* ctx, double* value);
/* What the communicator itself reports: *nranks_out (RCCL: ncclCommCount),
 * *rank_out (ncclCommUserRank); either may be NULL.  With bus_ids_out
 * non-NULL (on EVERY rank: it is then a collective) it receives each rank's
 * device PCI bus id (hipDeviceGetPCIBusId), CESS_BLS_BUS_ID_BYTES per rank in
 * rank order -- so a caller can show that N ranks ran on N distinct GPUs. */
int cess_bls_comm_info(cess_bls_ctx* ctx, int* nranks_out, int* rank_out, char* bus_ids_out);
/* "rccl", "shm" or "none" (static string). */
const char* cess_bls_comm_kind(cess_bls_ctx* ctx);

/* ---- host shared-memory transport ----
 * A fresh job name (POSIX shm name, NUL-terminated); create it on one rank and
 * distribute it out of band, like the RCCL id. */
int cess_bls_comm_shm_name(char name_out[CESS_BLS_COMM_NAME_BYTES]);
/* Attach the shared-memory transport to the context (collective: every rank
 * calls it with the same name; returns once all nranks are attached).  Waits
 * are bounded by env CESS_BLS_COMM_TIMEOUT_MS (default 300000): a rank that
 * times out fails with CESS_BLS_E_COMM and makes its peers fail too. */
int cess_bls_comm_init_shm(cess_bls_ctx* ctx, int nranks, int rank, const char* name);

/* Context-free communicator (no device needed): the merge step of the
 * sharded entry points for callers that verify their shards by other means
 * (e.g. keyed or device batches per rank), and for tests of the merge on
 * hosts without a GPU. */
typedef struct cess_bls_comm cess_bls_comm;
int cess_bls_comm_open_shm(const char* name, int nranks, int rank, cess_bls_comm** out);
void cess_bls_comm_close(cess_bls_comm* comm);
/* *agreed_out = the most negative status passed by any rank (0 if none failed). */
int cess_bls_comm_agree(cess_bls_comm* comm, int status, int* agreed_out);
/* shard_codes: this rank's shard (cess_bls_shard_range) of an n_total-record
 * batch; every rank receives the codes (n_total bytes, may be NULL) and the
 * bitmap (ceil(n_total/64) words, may be NULL) of the whole batch.  n_total
 * must be equal on every rank (else CESS_BLS_E_INVALID_ARG on all ranks). */
int cess_bls_comm_gather_verdicts(cess_bls_comm* comm, uint64_t n_total, const uint8_t* shard_codes,
                                  uint8_t* codes_out, uint64_t* bitmap_out);

/* ---- device memory on the context's GPU (for callers without a HIP runtime
 * of their own: keep a batch resident in HBM across device-resident calls) */
int cess_bls_device_alloc(cess_bls_ctx* ctx, size_t bytes, void** d_out);
int cess_bls_device_free(cess_bls_ctx* ctx, void* d);
int cess_bls_copy_to_device(cess_bls_ctx* ctx, void* d_dst, const void* src, size_t bytes);
int cess_bls_copy_from_device(cess_bls_ctx* ctx, void* dst, const void* d_src, size_t bytes);
int cess_bls_synchronize(cess_bls_ctx* ctx);

/* cp_enclave_verify::verify_bls(key, msg, sig) (primitives/enclave-verify/src/
 * lib.rs:230-235): NOTE the reversed argument order.  The key is decoded first
 * (PublicKey::deserialize(key).unwrap(), :231), then the signature (:233);
 * where the reference panics this returns CESS_BLS_E_BAD_KEY / _BAD_SIG
 * instead.  Otherwise CESS_BLS_OK with *ok_out = 1 iff puk.verify(msg, sig)
 * is Ok(()). */
int cess_bls_enclave_verify_bls(cess_bls_ctx* ctx, const uint8_t* key, size_t key_len, const uint8_t* msg,
                                size_t msg_len, const uint8_t* sig, size_t sig_len, int* ok_out);

/* ---- deserialize only (no pairing) ----
 * Signature::deserialize (src/lib.rs:138-152) for kind CESS_BLS_KIND_SIG, or
 * PublicKey::deserialize (src/lib.rs:68-82, including the G2 subgroup check)
 * for CESS_BLS_KIND_PK, over n encodings of any length (record i =
 * data[offsets[i] .. offsets[i+1])): codes_out[i] = 0, or SIG_LEN / SIG_POINT
 * (PK_LEN / PK_POINT).  Runs the decode kernels alone, so one call costs a
 * decode's latency, not a verification's.  Host buffers. */
#define CESS_BLS_KIND_SIG 0
#define CESS_BLS_KIND_PK 1
int cess_bls_deserialize_batch(cess_bls_ctx* ctx, int kind, size_t n, const uint8_t* data, const uint64_t* offsets,
                               uint8_t* codes_out);

/* ---- verdict cache (node host function + batcher) ----
 * Thread-safe map from a record -- SHA-256 over the length-prefixed (sig, msg,
 * key) bytes -- to its verdict code, bounded by `capacity` entries (at
 * capacity the oldest entries are evicted first, so memory stays bounded
 * whatever a transaction pool receives).  Only verdicts (codes 0..5) are ever
 * stored. */
#define CESS_BLS_CODE_UNAVAILABLE 0xff  /* no verdict: the caller's own path (e.g. the runtime's wasm verifier) decides */
typedef struct cess_bls_cache cess_bls_cache;
int cess_bls_cache_create(size_t capacity, cess_bls_cache** out);
void cess_bls_cache_destroy(cess_bls_cache* cache);
int cess_bls_cache_clear(cess_bls_cache* cache);
size_t cess_bls_cache_size(cess_bls_cache* cache);
/* Codes for n records of any lengths (layout of cess_bls_verify_batch_var):
 * cached records from the cache; the others (each distinct record once)
 * verified in ONE batch on ctx and inserted.  ctx NULL, or a batch that fails
 * (infrastructure): those records get CESS_BLS_CODE_UNAVAILABLE, nothing is
 * inserted, and the batch's status is returned (CESS_BLS_E_NO_DEVICE for
 * NULL) -- codes_out is filled in every case.  stats3 (may be NULL): cache
 * hits, records verified, entries evicted by this call. */
int cess_bls_cache_verify_var(cess_bls_cache* cache, cess_bls_ctx* ctx, size_t n, const uint8_t* sig_data,
                              const uint64_t* sig_offsets, const uint8_t* pk_data, const uint64_t* pk_offsets,
                              const uint8_t* msgs, const uint64_t* msg_offsets, uint8_t* codes_out,
                              uint64_t* stats3);
/* Insert verdicts obtained elsewhere (e.g. the gathered codes of a sharded
 * batch); codes must be verdicts (0..5). */
int cess_bls_cache_insert_var(cess_bls_cache* cache, size_t n, const uint8_t* sig_data, const uint64_t* sig_offsets,
                              const uint8_t* pk_data, const uint64_t* pk_offsets, const uint8_t* msgs,
                              const uint64_t* msg_offsets, const uint8_t* codes);
/* SHA-256 of the cache keys (exposed so callers and tests can check the key
 * derivation). */
int cess_bls_sha256(const uint8_t* data, size_t len, uint8_t out[32]);

/* Per-stage timings (ms, summed since the last reset) when CESS_BLS_F_PROFILE is
 * set.  names/ms arrays of length max; returns the number of stages. */
int cess_bls_stage_times(cess_bls_ctx* ctx, const char** names, double* ms, int max, int reset);
/* As cess_bls_stage_times, plus the number of kernel launches per stage
 * (launches may be NULL).  Each launch is bracketed by events on the stream it
 * runs on, so a stage's time is the sum of its own launch durations even when
 * the pipeline overlaps stages of different parts. */
int cess_bls_stage_stats(cess_bls_ctx* ctx, const char** names, double* ms, uint64_t* launches, int max, int reset);
/* Records per kernel launch (pipeline part): batches longer than this run as
 * parts whose decode/hash/prepare kernels overlap the previous part's Miller
 * loop on a second stream.  Default: max_batch (no overlap; overlap measured
 * slower on MI355X); env CESS_BLS_LAUNCH_RECORDS. */
uint64_t cess_bls_launch_records(cess_bls_ctx* ctx);

const char* cess_bls_status_string(int status);
const char* cess_bls_version(void);
/* HIP devices visible to this process (hipGetDeviceCount; 0 when there is no
 * device or the runtime fails).  Initialises the HIP runtime: a launcher that
 * must not touch the GPU counts devices some other way.  bench.py's ranks call
 * it before any context or communicator exists, so an N-rank job on a node
 * with fewer than N devices exits at once instead of meeting a peer-less
 * communicator (no reference counterpart: node-side launch plumbing). */
int cess_bls_device_count(void);

#ifdef __cplusplus
}
#endif
#endif /* CESS_BLS_H */
