// Internal declarations shared by the host translation units behind
// include/cess_bls.h (host.cpp: per-device context and the per-signature
// pipeline; host_rlc.cpp: RLC batch mode; host_multi.cpp: RCCL communicator,
// sharded batches and multi-device contexts).  Not part of the C ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <vector>

#include "../../include/cess_bls.h"
#include "../../include/cess_rsa.h"
#include "comm.hpp"
#include "kernels.hpp"

// kernels (k_*.hip)
__global__ void k_decode_sig(uint64_t, const uint8_t*, const uint8_t*, uint8_t*, uint8_t*, uint32_t*, uint64_t);
__global__ void k_decode_pk(uint64_t, const uint8_t*, const uint8_t*, uint8_t*, uint8_t*, uint32_t*, uint64_t, uint32_t);
__global__ void k_hash(uint64_t, const uint8_t*, const uint64_t*, const uint8_t*, uint32_t*, uint64_t);
__global__ void k_prepare(uint64_t, const uint32_t*, uint4*, uint64_t, uint8_t*, const uint8_t*);
__global__ void k_norm_lines(uint4*);
__global__ void k_miller(uint64_t, const uint8_t*, const uint8_t*, const uint32_t*, const uint32_t*, const uint32_t*,
                         const uint4*, uint4*, uint4*, uint64_t, const uint32_t*, uint64_t, const uint8_t*);
__global__ void k_miller2(uint64_t, const uint8_t*, const uint8_t*, const uint32_t*, const uint32_t*, const uint32_t*,
                          const uint4*, uint4*, uint4*, uint64_t, const uint32_t*, uint64_t, const uint8_t*);
__global__ void k_miller_rr(uint64_t, uint64_t, const uint8_t*, const uint8_t*, const uint32_t*, const uint4*, uint4*,
                            uint64_t, uint64_t);
__global__ void k_miller_rr2(uint64_t, uint64_t, const uint8_t*, const uint8_t*, const uint32_t*, const uint4*, uint4*,
                            uint64_t, uint64_t);
__global__ void k_norm_keys(uint64_t, uint64_t, uint4*, uint32_t*, uint8_t*);
__global__ void k_merge_pk(uint64_t, const uint32_t*, uint32_t, const uint8_t*, const uint8_t*, uint8_t*, uint8_t*);
__global__ void k_final(uint64_t, uint8_t*, uint4*, uint4*, uint64_t*, uint8_t*, uint64_t);
__global__ void k_final2(uint64_t, uint8_t*, uint4*, uint4*, uint64_t*, uint8_t*, uint64_t);
__global__ void k_keygen(uint64_t, const uint8_t*, uint8_t*);
__global__ void k_sign(uint64_t, const uint8_t*, const uint8_t*, const uint64_t*, uint8_t*);
__global__ void k_hash_out(uint64_t, const uint8_t*, const uint64_t*, uint8_t*);
// small-batch (latency) path (k_group.hip): one signature per wave
__global__ void k_group(uint64_t, const uint8_t*, const uint8_t*, const uint8_t*, const uint8_t*, const uint32_t*,
                        const uint32_t*, const uint32_t*, uint64_t, uint8_t*, uint8_t*);
__global__ void k_codes_bitmap(uint64_t, const uint8_t*, uint64_t*);
// RLC batch mode (k_rlc.hip)
__global__ void k_rlc_scale(uint64_t, const uint8_t*, const uint8_t*, const uint32_t*, const uint32_t*, const uint32_t*,
                            uint64_t, uint32_t*, uint32_t*, uint64_t, uint64_t, uint32_t);
__global__ void k_rlcd_scale(uint64_t, const uint8_t*, const uint8_t*, const uint32_t*, const uint32_t*, const uint32_t*,
                            uint64_t, uint32_t*, uint32_t*, uint64_t, uint64_t);
__global__ void k_gt_prod(uint32_t, const uint8_t*, uint4*, uint8_t*);
__global__ void k_g1_sum_segs(uint32_t, const uint64_t*, const uint64_t*, const uint32_t*, const uint32_t*, uint64_t,
                              uint32_t*, uint64_t);
__global__ void k_rlc_pairs_list(uint32_t, uint32_t, const uint32_t*, const uint32_t*, const uint32_t*, const uint8_t*, uint8_t*,
                                 uint8_t*, uint32_t*, uint32_t*, const uint32_t*);
__global__ void k_fp12_prod_segs(uint32_t, const uint32_t*, const uint4*, uint64_t, uint4*, uint4*);
__global__ void k_rlcd_records(uint64_t, const uint8_t*, const uint8_t*, const uint32_t*, uint64_t, uint32_t*, uint8_t*,
                               uint64_t);
__global__ void k_rlcd_s_records(uint32_t, const uint32_t*, uint8_t*, uint8_t*, uint32_t*);
__global__ void k_fp12_prod_chunks(uint32_t, const uint64_t*, const uint64_t*, const uint8_t*, const uint4*, uint64_t,
                                   uint4*);
__global__ void k_fp12_mul_each(uint32_t, uint4*, const uint4*);
__global__ void k_group_fe(uint32_t, const uint4*, uint8_t*, uint8_t*);
__global__ void k_msm_count(uint64_t, const uint8_t*, const uint8_t*, MsmSegs, const uint32_t*, uint64_t, uint32_t*);
__global__ void k_msm_scatter(uint64_t, const uint8_t*, const uint8_t*, MsmSegs, const uint32_t*, uint64_t, uint32_t*,
                              uint32_t*);
__global__ void k_inv_perm(uint64_t, const uint32_t*, uint32_t*);
__global__ void k_msm_aos(uint64_t, const uint32_t*, uint4*);
__global__ void k_msm_items(uint32_t, uint32_t, uint32_t, const uint32_t*, const uint32_t*, const uint32_t*, const uint32_t*,
                            const uint4*, const uint4*, uint32_t*, uint64_t);
__global__ void k_msm_bucket_sum(uint32_t, const uint32_t*, const uint32_t*, uint64_t, uint32_t*);
__global__ void k_msm_window(uint32_t, const uint32_t*, uint64_t, uint32_t*);
__global__ void k_msm_wsum(uint32_t, const uint32_t*, uint32_t*);
__global__ void k_msm_finish(uint32_t, uint32_t, const uint32_t*, uint32_t*, uint32_t*);

namespace cess_host {

enum Stage { ST_DECODE_SIG, ST_DECODE_PK, ST_HASH, ST_PREPARE, ST_MILLER, ST_FINAL, ST_RSA_CLASSIFY, ST_RSA_VERIFY,
             ST_GROUP, ST_SIGN, ST_N };
constexpr int kBlock = 256;

inline unsigned grid_for(uint64_t n) { return (unsigned)((n + kBlock - 1) / kBlock); }

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  int ensure(size_t want) {
    if (want <= bytes) return CESS_BLS_OK;
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
    if (hipMalloc(&p, want) != hipSuccess) return CESS_BLS_E_OOM;
    bytes = want;
    return CESS_BLS_OK;
  }
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
  template <class T>
  T* as() const {
    return static_cast<T*>(p);
  }
};

// State of one RLC batch between cess_bls_rlc_begin and cess_bls_rlc_finish.
struct RlcState {
  uint64_t n = 0;
  const uint8_t *sigs = nullptr, *pks = nullptr, *msgs = nullptr;   // caller's records (kept valid by the caller)
  const uint64_t* offs = nullptr;
  std::vector<uint8_t> codes;       // decode codes; 0 = candidate for the pairing check
  std::vector<uint32_t> perm;       // record indices sorted by key group
  std::vector<uint64_t> gbeg;       // K + 1 group boundaries in perm
  uint32_t K = 0;
  bool local_ok = false;
  // set only when the most recent rlc_begin completed: rlc_finish refuses
  // (CESS_BLS_E_INVALID_ARG) otherwise, so a failed or partial begin can never
  // be finished into "all verified" (fail closed)
  bool valid = false;
  bool per_sig = false;             // too many distinct keys for a combination: verified per signature
  uint64_t checks = 0, leaves = 0, leaf_sigs = 0;
  DevBuf P, Q, d_perm, d_seed, part, S, Qs, pk_in, pk_code, pk_inf, pk_aff, pk_coeffs, pk_usable;
  DevBuf rec_code, rec_inf, rec_sig, rec_h, rec_f, rec_f2, acc, slots, fin_code, fin_bm, gt, gts, tmp;
  DevBuf seg, part2, rec_coeffs, lists, d_gt_all;
  // distinct-key RLC (CESS_BLS_F_RLC_DISTINCT): every record's Miller value
  // f_i (stride n), the chunk-product ping-pong arrays and chunk bounds
  bool distinct = false;
  DevBuf d_rec_f, pr_a, pr_b, pr_lo, pr_hi;
  // bucket sums of the first check (k_msm_*): records' affine points and codes
  // for the whole batch (SoA stride n), group ids, bucket tables
  bool pts = false;                 // the batch's points are kept on the device (bucket sums possible)
  bool pq = false;                  // P, Q (per-record multiples) computed
  bool aos = false, have_pos = false;
  uint64_t index_hi = 0;            // scalar index base of this batch (rlc_begin_at)
  DevBuf Xs, Xh, Xsa, Xha, d_pos, m_bounds, d_code, d_inf, d_grp, m_cnt, m_start, m_cur, m_items, m_idx, m_part, m_bsum, m_T, m_U;
};

// Stage buffers of one in-flight pipeline part (SoA, stride = qcap).
struct StageSlot {
  DevBuf inf, sig_aff, h_aff, pk_aff, coeffs;
};

// One profiled kernel launch: [a, b] events on the launch's stream.
struct ProfRec {
  int stage;
  hipEvent_t a, b;
};

}  // namespace cess_host

struct RsaState;   // host_rsa.cpp
void cess_rsa_state_free(cess_bls_ctx* c);

struct cess_bls_ctx {
  int device = 0;
  uint64_t cap = 0;    // records per host-API chunk (staging buffers)
  uint64_t qcap = 0;   // records per kernel launch (pipeline part; stage-buffer stride)
  uint64_t small = 0;  // batches of at most this many records take the lane-group path (k_group)
  uint32_t flags = 0;
  uint32_t mode = CESS_BLS_MODE_PER_SIG;
  hipStream_t stream = nullptr;
  // Pipeline (run_chunk): a chunk longer than qcap runs as parts; the light
  // kernels of part i+1 (decode, hash, prepare: no LDS, 128 VGPRs) run on
  // stream2 while k_miller of part i (one wave per SIMD: 144 KiB of LDS, 256
  // VGPRs) runs on the launch stream, so they share the CUs' issue slots.
  // Two stage slots alternate between parts.
  hipStream_t stream2 = nullptr;
  // small-batch path: the key decode (stream2) and hashing (stream3) run
  // beside the signature decode; the key decode's codes go to code2/inf2
  hipStream_t stream3 = nullptr;
  cess_host::DevBuf code2, inf2;
  hipEvent_t ev_start = nullptr, ev_light[2] = {}, ev_mill[2] = {};
  cess_host::StageSlot slot[2];
  cess_host::DevBuf pre, code, fval, fe_slots, bitmap, neg_g2;
  // staging for the host-buffer APIs
  cess_host::DevBuf in_sigs, in_pks, in_msgs, in_offs, out_gt, in_sks, out_bytes;
  // profiling: per-launch events (pool reused after each collect)
  std::vector<hipEvent_t> evpool;
  size_t evused = 0;
  std::vector<cess_host::ProfRec> prof;
  double stage_ms[cess_host::ST_N] = {};
  uint64_t stage_launches[cess_host::ST_N] = {};
  cess_host::RlcState* rlc = nullptr;
  // distinct-key table (cess_bls_keys_load): decoded keys + G2Prepared rows, stride = nkeys
  uint32_t nkeys = 0;
  cess_host::DevBuf key_in, key_code, key_inf, key_aff, key_coeffs, in_idx;
  // per key: 1 if its lines were normalised to c2 = 1 (k_norm_keys)
  cess_host::DevBuf key_norm;
  // ordering of successive calls on possibly different streams: every entry
  // point waits for the previous call's work (done_ev on last_stream)
  hipEvent_t done_ev = nullptr;
  hipStream_t last_stream = nullptr;
  bool pending = false;
  // one host thread at a time (the ABI contract); a second concurrent caller
  // gets CESS_BLS_E_BUSY instead of racing on the context buffers
  std::mutex busy;
  // communicator of the sharded entry points (comm.hpp): RCCL
  // (cess_bls_comm_init, one rank per process and GPU) or host shared memory
  // (cess_bls_comm_init_shm); owned
  cess_host::Transport* xport = nullptr;
  int nranks = 1, rank = 0;
  cess_host::DevBuf comm_buf, comm_words, comm_codes;
  // multi-device context (cess_bls_config.n_devices > 1): one sub-context per
  // device, batches sharded by index across them from host threads
  std::vector<cess_bls_ctx*> subs;
  // RSA PKCS#1 v1.5 key tables and staging (host_rsa.cpp)
  RsaState* rsa = nullptr;
};

#define HIPCHK(x)                                 \
  do {                                            \
    if ((x) != hipSuccess) return CESS_BLS_E_HIP; \
  } while (0)

namespace cess_host {

// RAII guard for the one-thread-at-a-time contract
struct CtxLock {
  std::unique_lock<std::mutex> lk;
  explicit CtxLock(cess_bls_ctx* c) : lk(c->busy, std::try_to_lock) {}
  bool ok() const { return lk.owns_lock(); }
};

// make stream s wait for the previous call's work; called by every entry point
// before it enqueues anything (the context buffers are shared across calls)
int order_begin(cess_bls_ctx* c, hipStream_t s);
// record the end of this call's work on s
int order_end(cess_bls_ctx* c, hipStream_t s);

// profiling brackets around one launch on stream s (no-ops without CESS_BLS_F_PROFILE)
int prof_begin(cess_bls_ctx* c, hipStream_t s, int stage, hipEvent_t* a);
int prof_end(cess_bls_ctx* c, hipStream_t s, int stage, hipEvent_t a);
int run_chunk(cess_bls_ctx* c, hipStream_t s, uint64_t n, const uint8_t* sigs, const uint8_t* pks, const uint8_t* msgs,
              const uint64_t* offs, const uint8_t* pre, uint8_t* codes, uint64_t* bitmap, uint8_t* gt);
int verify_host(cess_bls_ctx* c, size_t n, const uint8_t* sigs, const uint8_t* pks, const uint8_t* msgs,
                const uint64_t* offs, const uint8_t* pre, uint8_t* codes_out, uint64_t* bitmap_out, uint8_t* gt_out);
int verify_var_host(cess_bls_ctx* c, size_t n, const uint8_t* sig_data, const uint64_t* sig_offsets,
                    const uint8_t* pk_data, const uint64_t* pk_offsets, const uint8_t* msgs, const uint64_t* msg_offsets,
                    uint8_t* codes_out, uint64_t* bitmap_out);
int collect_profile(cess_bls_ctx* c, hipStream_t s);
// RLC (host_rlc.cpp)
int rlc_begin(cess_bls_ctx* c, size_t n, const uint8_t* sigs, const uint8_t* pks, const uint8_t* msgs,
              const uint64_t* offs, const uint8_t* seed32, uint8_t* gt_out);
// index_hi: added to every record index of the scalar derivation (shard k
// passes k << 40, so shards never share an r_i under one seed)
int rlc_begin_at(cess_bls_ctx* c, size_t n, const uint8_t* sigs, const uint8_t* pks, const uint8_t* msgs,
                 const uint64_t* offs, const uint8_t* seed32, uint64_t index_hi, uint8_t* gt_out);
int rlc_finish(cess_bls_ctx* c, uint8_t* codes_out, uint64_t* bitmap_out, uint64_t* stats4);
int gt_product_is_one(cess_bls_ctx* c, size_t m, const uint8_t* gts, bool gts_on_device, int* is_one);
int verify_rlc_host(cess_bls_ctx* c, size_t n, const uint8_t* sigs, const uint8_t* pks, const uint8_t* msgs,
                    const uint64_t* offs, const uint8_t* seed32, uint8_t* codes_out, uint64_t* bitmap_out,
                    uint64_t* stats4);
// OS randomness for RLC seeds drawn by the library (mode = RLC)
int os_random(uint8_t* out, size_t n);
// bitmap words from codes (host)
void bitmap_from_codes(const uint8_t* codes, uint64_t n, uint64_t* words);

}  // namespace cess_host
