// Host runtime behind include/cess_bls.h: one context per GPU, a HIP stream,
// device stage buffers sized for one launch chunk, and the constant
// G2PREPARED_NEG_G table (reference src/lib.rs:19-21) built once on the device.
//
// There is no CPU compute path: every verdict is produced by the gfx950 kernels.
// Without a usable HIP device, cess_bls_ctx_create fails with CESS_BLS_E_NO_DEVICE.
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "../../include/cess_bls.h"
#include "bls/consts.hpp"
#include "kernels.hpp"

// kernels (k_*.hip)
__global__ void k_decode_sig(uint64_t, const uint8_t*, const uint8_t*, uint8_t*, uint8_t*, uint32_t*, uint64_t);
__global__ void k_decode_pk(uint64_t, const uint8_t*, const uint8_t*, uint8_t*, uint8_t*, uint32_t*, uint64_t);
__global__ void k_hash(uint64_t, const uint8_t*, const uint64_t*, const uint8_t*, uint32_t*, uint64_t);
__global__ void k_prepare(uint64_t, const uint32_t*, uint4*, uint64_t);
__global__ void k_miller(uint64_t, const uint8_t*, const uint8_t*, const uint32_t*, const uint32_t*, const uint32_t*,
                         const uint4*, uint4*, uint4*, uint64_t, const uint32_t*, uint64_t);
__global__ void k_merge_pk(uint64_t, const uint32_t*, const uint8_t*, const uint8_t*, uint8_t*, uint8_t*);
__global__ void k_final(uint64_t, uint8_t*, uint4*, uint4*, uint64_t*, uint8_t*, uint64_t);
__global__ void k_keygen(uint64_t, const uint8_t*, uint8_t*);
__global__ void k_sign(uint64_t, const uint8_t*, const uint8_t*, const uint64_t*, uint8_t*);
__global__ void k_hash_out(uint64_t, const uint8_t*, const uint64_t*, uint8_t*);
// RLC batch mode (k_rlc.hip)
__global__ void k_rlc_scale(uint64_t, const uint8_t*, const uint8_t*, const uint32_t*, const uint32_t*, const uint32_t*,
                            uint64_t, uint32_t*, uint32_t*, uint64_t, uint64_t);
__global__ void k_g1_sum(uint64_t, const uint32_t*, uint64_t, const uint32_t*, uint64_t, uint32_t*, uint64_t);
__global__ void k_rlc_pairs(uint32_t, const uint32_t*, const uint32_t*, uint64_t, const uint8_t*, uint8_t*, uint8_t*,
                            uint32_t*, uint32_t*);
__global__ void k_fp12_prod(uint32_t, const uint4*, uint64_t, uint4*);
__global__ void k_gt_prod(uint32_t, const uint8_t*, uint4*, uint8_t*);
__global__ void k_g1_sum_segs(const uint64_t*, const uint64_t*, const uint32_t*, const uint32_t*, uint64_t, uint32_t*,
                              uint64_t);
__global__ void k_rlc_pairs_multi(uint32_t, uint32_t, const uint32_t*, const uint32_t*, const uint8_t*, uint8_t*,
                                  uint8_t*, uint32_t*, uint32_t*);
__global__ void k_rep_rows(uint32_t, uint32_t, uint32_t, const uint4*, uint4*);
__global__ void k_fp12_prod_multi(uint32_t, uint32_t, const uint4*, uint4*);

namespace {

enum Stage { ST_DECODE_SIG, ST_DECODE_PK, ST_HASH, ST_PREPARE, ST_MILLER, ST_FINAL, ST_N };
const char* kStageNames[ST_N] = {"k_decode_sig", "k_decode_pk", "k_hash", "k_prepare", "k_miller", "k_final"};
constexpr int kBlock = 256;

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
  uint64_t checks = 0, leaves = 0, leaf_sigs = 0;
  DevBuf P, Q, d_perm, d_seed, part, S, Qs, pk_in, pk_code, pk_inf, pk_aff, pk_coeffs, pk_usable;
  DevBuf rec_code, rec_inf, rec_sig, rec_h, rec_f, rec_f2, acc, slots, fin_code, fin_bm, gt, gts, tmp;
  DevBuf seg, part2, rec_coeffs;
};

}  // namespace

struct cess_bls_ctx {
  int device = 0;
  uint64_t cap = 0;
  uint32_t flags = 0;
  hipStream_t stream = nullptr;
  // stage buffers (SoA, stride = cap)
  DevBuf pre, code, inf, sig_aff, pk_aff, h_aff, coeffs, fval, fe_slots, bitmap, neg_g2;
  // staging for the host-buffer APIs
  DevBuf in_sigs, in_pks, in_msgs, in_offs, out_gt, in_sks, out_bytes;
  std::vector<uint8_t> h_pre;
  // profiling
  hipEvent_t ev[ST_N + 1] = {};
  double stage_ms[ST_N] = {};
  RlcState* rlc = nullptr;
  // distinct-key table (cess_bls_keys_load): decoded keys + G2Prepared rows, stride = nkeys
  uint32_t nkeys = 0;
  DevBuf key_in, key_code, key_inf, key_aff, key_coeffs, in_idx;
};

#define HIPCHK(x)                          \
  do {                                     \
    if ((x) != hipSuccess) return CESS_BLS_E_HIP; \
  } while (0)

static inline unsigned grid_for(uint64_t n) { return (unsigned)((n + kBlock - 1) / kBlock); }


extern "C" const char* cess_bls_version(void) { return "cess_amd-bls 0.1 (gfx950)"; }

extern "C" const char* cess_bls_status_string(int s) {
  switch (s) {
    case CESS_BLS_OK: return "ok";
    case CESS_BLS_E_INVALID_ARG: return "invalid argument";
    case CESS_BLS_E_NO_DEVICE: return "no HIP device (the verifier has no CPU fallback)";
    case CESS_BLS_E_HIP: return "HIP runtime error";
    case CESS_BLS_E_OOM: return "device out of memory";
    case CESS_BLS_E_RCCL: return "RCCL error";
  }
  return "unknown status";
}

static int alloc_stage(cess_bls_ctx* c) {
  uint64_t n = c->cap;
  int r = CESS_BLS_OK;
  r |= c->pre.ensure(n);
  r |= c->code.ensure(n);
  r |= c->inf.ensure(n);
  r |= c->sig_aff.ensure(n * CESS_W_G1 * 4);
  r |= c->h_aff.ensure(n * CESS_W_G1 * 4);
  r |= c->fval.ensure(n * CESS_W_FP12 * 4);
  r |= c->fe_slots.ensure(n * CESS_W_FP12 * 4 * CESS_FE_SLOTS);
  r |= c->bitmap.ensure((n / 64 + 1) * 8);
  return r ? CESS_BLS_E_OOM : CESS_BLS_OK;
}

extern "C" int cess_bls_ctx_create(const cess_bls_config* cfg, cess_bls_ctx** out) {
  if (!out) return CESS_BLS_E_INVALID_ARG;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return CESS_BLS_E_NO_DEVICE;
  cess_bls_ctx* c = new cess_bls_ctx();
  c->device = (cfg && cfg->device >= 0) ? cfg->device : 0;
  if (c->device < 0 || c->device >= ndev) {
    delete c;
    return CESS_BLS_E_INVALID_ARG;
  }
  uint64_t cap = (cfg && cfg->max_batch) ? cfg->max_batch : (1ull << 20);
  c->cap = (cap + 63) & ~63ull;
  c->flags = cfg ? cfg->flags : 0;
  if (hipSetDevice(c->device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return CESS_BLS_E_HIP;
  }
  int r = alloc_stage(c);
  if (r == CESS_BLS_OK) r = c->neg_g2.ensure(CESS_W_COEFFS * 4);
  if (r != CESS_BLS_OK) {
    cess_bls_ctx_destroy(c);
    return r;
  }
  for (int i = 0; i <= ST_N; i++)
    if (hipEventCreate(&c->ev[i]) != hipSuccess) {
      cess_bls_ctx_destroy(c);
      return CESS_BLS_E_HIP;
    }
  // G2PREPARED_NEG_G: prepare -G2 on the device with the same kernel (n = 1, stride = 1)
  uint32_t aff[48];
  {
    using namespace bls::c;
    const uint32_t* src[4] = {G2_GEN_X0, G2_GEN_X1, G2_GEN_Y0, G2_GEN_Y1};
    for (int j = 0; j < 4; j++) memcpy(aff + 12 * j, src[j], 48);
    // negate y (Montgomery values are < p): y -> p - y, per Fp component
    for (int j = 2; j < 4; j++) {
      uint64_t borrow = 0;
      for (int k = 0; k < 12; k++) {
        uint64_t d = (uint64_t)P_RAW[k] - aff[12 * j + k] - borrow;
        aff[12 * j + k] = (uint32_t)d;
        borrow = (d >> 63) & 1;
      }
    }
  }
  DevBuf tmp;
  if (tmp.ensure(sizeof(aff)) != CESS_BLS_OK || hipMemcpy(tmp.p, aff, sizeof(aff), hipMemcpyHostToDevice) != hipSuccess) {
    cess_bls_ctx_destroy(c);
    return CESS_BLS_E_HIP;
  }
  hipLaunchKernelGGL(k_prepare, dim3(1), dim3(64), 0, c->stream, (uint64_t)1, tmp.as<uint32_t>(), c->neg_g2.as<uint4>(),
                     (uint64_t)1);
  if (hipGetLastError() != hipSuccess || hipStreamSynchronize(c->stream) != hipSuccess) {
    cess_bls_ctx_destroy(c);
    return CESS_BLS_E_HIP;
  }
  *out = c;
  return CESS_BLS_OK;
}

extern "C" void cess_bls_ctx_destroy(cess_bls_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  for (int i = 0; i <= ST_N; i++)
    if (c->ev[i]) (void)hipEventDestroy(c->ev[i]);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c->rlc;
  delete c;
}

// Enqueue the verification pipeline for one chunk of n <= cap records.
// sigs/pks/msgs/offs/codes/bitmap/pre are device pointers; gt (optional).
static int run_chunk(cess_bls_ctx* c, hipStream_t s, uint64_t n, const uint8_t* sigs, const uint8_t* pks,
                     const uint8_t* msgs, const uint64_t* offs, const uint8_t* pre, uint8_t* codes, uint64_t* bitmap,
                     uint8_t* gt) {
  const uint64_t st = c->cap;
  // per-record key buffers (19.6 KB of line coefficients per signature) are
  // allocated on first use: keyed batches never touch them
  if (c->pk_aff.ensure(st * CESS_W_G2 * 4) | c->coeffs.ensure(st * (uint64_t)CESS_W_COEFFS * 4)) return CESS_BLS_E_OOM;
  const bool prof = (c->flags & CESS_BLS_F_PROFILE) != 0;
  const unsigned g = grid_for(n);
  uint8_t* inf = c->inf.as<uint8_t>();
  if (prof) HIPCHK(hipEventRecord(c->ev[0], s));
  hipLaunchKernelGGL(k_decode_sig, dim3(g), dim3(kBlock), 0, s, n, sigs, pre, codes, inf, c->sig_aff.as<uint32_t>(), st);
  if (prof) HIPCHK(hipEventRecord(c->ev[1], s));
  hipLaunchKernelGGL(k_decode_pk, dim3(g), dim3(kBlock), 0, s, n, pks, pre, codes, inf, c->pk_aff.as<uint32_t>(), st);
  if (prof) HIPCHK(hipEventRecord(c->ev[2], s));
  hipLaunchKernelGGL(k_hash, dim3(g), dim3(kBlock), 0, s, n, msgs, offs, (const uint8_t*)codes, c->h_aff.as<uint32_t>(), st);
  if (prof) HIPCHK(hipEventRecord(c->ev[3], s));
  hipLaunchKernelGGL(k_prepare, dim3(g), dim3(kBlock), 0, s, n, (const uint32_t*)c->pk_aff.as<uint32_t>(),
                     c->coeffs.as<uint4>(), st);
  if (prof) HIPCHK(hipEventRecord(c->ev[4], s));
  hipLaunchKernelGGL(k_miller, dim3(g), dim3(kBlock), 0, s, n, (const uint8_t*)codes, (const uint8_t*)inf,
                     (const uint32_t*)c->sig_aff.as<uint32_t>(), (const uint32_t*)c->h_aff.as<uint32_t>(),
                     (const uint32_t*)c->neg_g2.as<uint32_t>(), (const uint4*)c->coeffs.as<uint4>(),
                     c->fval.as<uint4>(), c->fe_slots.as<uint4>(), st, (const uint32_t*)nullptr, st);
  if (prof) HIPCHK(hipEventRecord(c->ev[5], s));
  hipLaunchKernelGGL(k_final, dim3(g), dim3(kBlock), 0, s, n, codes, c->fval.as<uint4>(), c->fe_slots.as<uint4>(), bitmap,
                     gt, st);
  if (prof) HIPCHK(hipEventRecord(c->ev[6], s));
  HIPCHK(hipGetLastError());
  return CESS_BLS_OK;
}

static int collect_profile(cess_bls_ctx* c, hipStream_t s) {
  if (!(c->flags & CESS_BLS_F_PROFILE)) return CESS_BLS_OK;
  HIPCHK(hipStreamSynchronize(s));
  for (int i = 0; i < ST_N; i++) {
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, c->ev[i], c->ev[i + 1]));
    c->stage_ms[i] += ms;
  }
  return CESS_BLS_OK;
}

// Host-buffer batch over fixed-stride inputs (pre: optional host pre-flags)
static int verify_host(cess_bls_ctx* c, size_t n, const uint8_t* sigs, const uint8_t* pks, const uint8_t* msgs,
                       const uint64_t* offs, const uint8_t* pre, uint8_t* codes_out, uint64_t* bitmap_out,
                       uint8_t* gt_out) {
  if (n == 0) return CESS_BLS_OK;
  if (!sigs || !pks || !offs || (!msgs && offs[n] != offs[0])) return CESS_BLS_E_INVALID_ARG;
  HIPCHK(hipSetDevice(c->device));
  hipStream_t s = c->stream;
  std::vector<uint64_t> rebased;
  std::vector<uint64_t> words;
  for (size_t off = 0; off < n; off += c->cap) {
    uint64_t m = std::min<uint64_t>(c->cap, n - off);
    uint64_t mb0 = offs[off], mb1 = offs[off + m];
    if (mb1 < mb0) return CESS_BLS_E_INVALID_ARG;
    rebased.resize(m + 1);
    for (uint64_t j = 0; j <= m; j++) {
      if (j && offs[off + j] < offs[off + j - 1]) return CESS_BLS_E_INVALID_ARG;
      rebased[j] = offs[off + j] - mb0;
    }
    int r = CESS_BLS_OK;
    r |= c->in_sigs.ensure(m * 48);
    r |= c->in_pks.ensure(m * 96);
    r |= c->in_msgs.ensure(std::max<uint64_t>(mb1 - mb0, 1));
    r |= c->in_offs.ensure((m + 1) * 8);
    if (gt_out) r |= c->out_gt.ensure(m * 576);
    if (r) return CESS_BLS_E_OOM;
    HIPCHK(hipMemcpyAsync(c->in_sigs.p, sigs + 48 * off, m * 48, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(c->in_pks.p, pks + 96 * off, m * 96, hipMemcpyHostToDevice, s));
    if (mb1 > mb0) HIPCHK(hipMemcpyAsync(c->in_msgs.p, msgs + mb0, mb1 - mb0, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(c->in_offs.p, rebased.data(), (m + 1) * 8, hipMemcpyHostToDevice, s));
    const uint8_t* dpre = nullptr;
    if (pre) {
      HIPCHK(hipMemcpyAsync(c->pre.p, pre + off, m, hipMemcpyHostToDevice, s));
      dpre = c->pre.as<uint8_t>();
    }
    if (gt_out) HIPCHK(hipMemsetAsync(c->out_gt.p, 0, m * 576, s));
    r = run_chunk(c, s, m, c->in_sigs.as<uint8_t>(), c->in_pks.as<uint8_t>(), c->in_msgs.as<uint8_t>(),
                  c->in_offs.as<uint64_t>(), dpre, c->code.as<uint8_t>(), c->bitmap.as<uint64_t>(),
                  gt_out ? c->out_gt.as<uint8_t>() : nullptr);
    if (r) return r;
    if (codes_out) HIPCHK(hipMemcpyAsync(codes_out + off, c->code.p, m, hipMemcpyDeviceToHost, s));
    if (gt_out) HIPCHK(hipMemcpyAsync(gt_out + 576 * off, c->out_gt.p, m * 576, hipMemcpyDeviceToHost, s));
    uint64_t nw = (m + 63) / 64;
    words.resize(nw);
    HIPCHK(hipMemcpyAsync(words.data(), c->bitmap.p, nw * 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (bitmap_out) memcpy(bitmap_out + off / 64, words.data(), nw * 8);
    r = collect_profile(c, s);
    if (r) return r;
  }
  return CESS_BLS_OK;
}

extern "C" int cess_bls_verify_batch(cess_bls_ctx* c, size_t n, const uint8_t* sigs, const uint8_t* pks,
                                     const uint8_t* msgs, const uint64_t* msg_offsets, uint8_t* codes_out,
                                     uint64_t* bitmap_out) {
  if (!c) return CESS_BLS_E_INVALID_ARG;
  return verify_host(c, n, sigs, pks, msgs, msg_offsets, nullptr, codes_out, bitmap_out, nullptr);
}

extern "C" int cess_bls_gt_batch(cess_bls_ctx* c, size_t n, const uint8_t* sigs, const uint8_t* pks, const uint8_t* msgs,
                                 const uint64_t* msg_offsets, uint8_t* codes_out, uint8_t* gt_out) {
  if (!c || !gt_out) return CESS_BLS_E_INVALID_ARG;
  return verify_host(c, n, sigs, pks, msgs, msg_offsets, nullptr, codes_out, nullptr, gt_out);
}

extern "C" int cess_bls_verify_batch_var(cess_bls_ctx* c, size_t n, const uint8_t* sig_data, const uint64_t* sig_offsets,
                                         const uint8_t* pk_data, const uint64_t* pk_offsets, const uint8_t* msgs,
                                         const uint64_t* msg_offsets, uint8_t* codes_out, uint64_t* bitmap_out) {
  if (!c || !sig_offsets || !pk_offsets || !msg_offsets) return CESS_BLS_E_INVALID_ARG;
  if (n == 0) return CESS_BLS_OK;
  std::vector<uint8_t> sigs(n * 48, 0), pks(n * 96, 0), pre(n, 0);
  for (size_t i = 0; i < n; i++) {
    uint64_t sl = sig_offsets[i + 1] - sig_offsets[i], pl = pk_offsets[i + 1] - pk_offsets[i];
    if (sig_offsets[i + 1] < sig_offsets[i] || pk_offsets[i + 1] < pk_offsets[i]) return CESS_BLS_E_INVALID_ARG;
    if (sl == 48) memcpy(&sigs[48 * i], sig_data + sig_offsets[i], 48);
    else pre[i] |= PRE_SIG_LEN_BAD;
    if (pl == 96) memcpy(&pks[96 * i], pk_data + pk_offsets[i], 96);
    else pre[i] |= PRE_PK_LEN_BAD;
  }
  return verify_host(c, n, sigs.data(), pks.data(), msgs, msg_offsets, pre.data(), codes_out, bitmap_out, nullptr);
}

extern "C" int cess_bls_verify(cess_bls_ctx* c, const uint8_t* sig, size_t sig_len, const uint8_t* msg, size_t msg_len,
                               const uint8_t* key, size_t key_len, uint8_t* code_out) {
  if (!c || !code_out || (!sig && sig_len) || (!key && key_len) || (!msg && msg_len)) return CESS_BLS_E_INVALID_ARG;
  uint64_t so[2] = {0, sig_len}, po[2] = {0, key_len}, mo[2] = {0, msg_len};
  static const uint8_t zero = 0;
  return cess_bls_verify_batch_var(c, 1, sig ? sig : &zero, so, key ? key : &zero, po, msg ? msg : &zero, mo, code_out,
                                   nullptr);
}

extern "C" int cess_bls_verify_batch_device(cess_bls_ctx* c, size_t n, const uint8_t* d_sigs, const uint8_t* d_pks,
                                            const uint8_t* d_msgs, const uint64_t* d_offs, uint8_t* d_codes,
                                            uint64_t* d_bitmap, void* stream) {
  if (!c || !d_sigs || !d_pks || !d_offs || !d_codes) return CESS_BLS_E_INVALID_ARG;
  HIPCHK(hipSetDevice(c->device));
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  for (size_t off = 0; off < n; off += c->cap) {
    uint64_t m = std::min<uint64_t>(c->cap, n - off);
    int r = run_chunk(c, s, m, d_sigs + 48 * off, d_pks + 96 * off, d_msgs, d_offs + off, nullptr, d_codes + off,
                      d_bitmap ? d_bitmap + off / 64 : c->bitmap.as<uint64_t>(), nullptr);
    if (r) return r;
    if (c->flags & CESS_BLS_F_PROFILE) {
      r = collect_profile(c, s);
      if (r) return r;
    }
  }
  return CESS_BLS_OK;
}

// distinct-key table ---------------------------------------------------------
// Per-key work of PublicKey::deserialize (src/lib.rs:68-82) and
// G2Prepared::from (:88) done once per distinct key (SURVEY §8(a) A5/A11:
// "cacheable per distinct pk"); the keyed batches then index the table.
extern "C" int cess_bls_keys_load(cess_bls_ctx* c, size_t k, const uint8_t* pks, uint8_t* key_codes_out) {
  if (!c || (k && !pks) || k > 0xffffffffull) return CESS_BLS_E_INVALID_ARG;
  HIPCHK(hipSetDevice(c->device));
  hipStream_t s = c->stream;
  c->nkeys = 0;
  if (k == 0) return CESS_BLS_OK;
  int r = c->key_in.ensure(k * 96) | c->key_code.ensure(k) | c->key_inf.ensure(k) |
          c->key_aff.ensure(k * CESS_W_G2 * 4) | c->key_coeffs.ensure(k * (uint64_t)CESS_W_COEFFS * 4);
  if (r) return CESS_BLS_E_OOM;
  HIPCHK(hipMemcpyAsync(c->key_in.p, pks, k * 96, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemsetAsync(c->key_code.p, 0, k, s));
  HIPCHK(hipMemsetAsync(c->key_inf.p, 0, k, s));
  hipLaunchKernelGGL(k_decode_pk, dim3(grid_for(k)), dim3(kBlock), 0, s, (uint64_t)k, c->key_in.as<uint8_t>(),
                     (const uint8_t*)nullptr, c->key_code.as<uint8_t>(), c->key_inf.as<uint8_t>(),
                     c->key_aff.as<uint32_t>(), (uint64_t)k);
  hipLaunchKernelGGL(k_prepare, dim3(grid_for(k)), dim3(kBlock), 0, s, (uint64_t)k,
                     (const uint32_t*)c->key_aff.as<uint32_t>(), c->key_coeffs.as<uint4>(), (uint64_t)k);
  HIPCHK(hipGetLastError());
  if (key_codes_out) HIPCHK(hipMemcpyAsync(key_codes_out, c->key_code.p, k, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  c->nkeys = (uint32_t)k;
  return CESS_BLS_OK;
}

// One chunk of a keyed batch: sig decode, key verdicts from the table, hash,
// Miller loop over the table's coefficient rows, final exponentiation.
static int run_chunk_keyed(cess_bls_ctx* c, hipStream_t s, uint64_t n, const uint8_t* sigs, const uint32_t* idx,
                           const uint8_t* msgs, const uint64_t* offs, uint8_t* codes, uint64_t* bitmap) {
  const uint64_t st = c->cap;
  const bool prof = (c->flags & CESS_BLS_F_PROFILE) != 0;
  const unsigned g = grid_for(n);
  uint8_t* inf = c->inf.as<uint8_t>();
  if (prof) HIPCHK(hipEventRecord(c->ev[0], s));
  hipLaunchKernelGGL(k_decode_sig, dim3(g), dim3(kBlock), 0, s, n, sigs, (const uint8_t*)nullptr, codes, inf,
                     c->sig_aff.as<uint32_t>(), st);
  if (prof) HIPCHK(hipEventRecord(c->ev[1], s));
  hipLaunchKernelGGL(k_merge_pk, dim3(g), dim3(kBlock), 0, s, n, idx, (const uint8_t*)c->key_code.as<uint8_t>(),
                     (const uint8_t*)c->key_inf.as<uint8_t>(), codes, inf);
  if (prof) HIPCHK(hipEventRecord(c->ev[2], s));
  hipLaunchKernelGGL(k_hash, dim3(g), dim3(kBlock), 0, s, n, msgs, offs, (const uint8_t*)codes, c->h_aff.as<uint32_t>(), st);
  if (prof) HIPCHK(hipEventRecord(c->ev[3], s));
  if (prof) HIPCHK(hipEventRecord(c->ev[4], s));
  hipLaunchKernelGGL(k_miller, dim3(g), dim3(kBlock), 0, s, n, (const uint8_t*)codes, (const uint8_t*)inf,
                     (const uint32_t*)c->sig_aff.as<uint32_t>(), (const uint32_t*)c->h_aff.as<uint32_t>(),
                     (const uint32_t*)c->neg_g2.as<uint32_t>(), (const uint4*)c->key_coeffs.as<uint4>(),
                     c->fval.as<uint4>(), c->fe_slots.as<uint4>(), st, idx, (uint64_t)c->nkeys);
  if (prof) HIPCHK(hipEventRecord(c->ev[5], s));
  hipLaunchKernelGGL(k_final, dim3(g), dim3(kBlock), 0, s, n, codes, c->fval.as<uint4>(), c->fe_slots.as<uint4>(), bitmap,
                     (uint8_t*)nullptr, st);
  if (prof) HIPCHK(hipEventRecord(c->ev[6], s));
  HIPCHK(hipGetLastError());
  return CESS_BLS_OK;
}

extern "C" int cess_bls_verify_batch_keyed_device(cess_bls_ctx* c, size_t n, const uint8_t* d_sigs,
                                                  const uint32_t* d_key_idx, const uint8_t* d_msgs,
                                                  const uint64_t* d_offs, uint8_t* d_codes, uint64_t* d_bitmap,
                                                  void* stream) {
  if (!c || !d_sigs || !d_key_idx || !d_offs || !d_codes) return CESS_BLS_E_INVALID_ARG;
  if (n == 0) return CESS_BLS_OK;
  if (c->nkeys == 0) return CESS_BLS_E_INVALID_ARG;
  HIPCHK(hipSetDevice(c->device));
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  for (size_t off = 0; off < n; off += c->cap) {
    uint64_t m = std::min<uint64_t>(c->cap, n - off);
    int r = run_chunk_keyed(c, s, m, d_sigs + 48 * off, d_key_idx + off, d_msgs, d_offs + off, d_codes + off,
                            d_bitmap ? d_bitmap + off / 64 : c->bitmap.as<uint64_t>());
    if (r) return r;
    r = collect_profile(c, s);
    if (r) return r;
  }
  return CESS_BLS_OK;
}

extern "C" int cess_bls_verify_batch_keyed(cess_bls_ctx* c, size_t n, const uint8_t* sigs, const uint32_t* key_idx,
                                           const uint8_t* msgs, const uint64_t* offs, uint8_t* codes_out,
                                           uint64_t* bitmap_out) {
  if (!c) return CESS_BLS_E_INVALID_ARG;
  if (n == 0) return CESS_BLS_OK;
  if (!sigs || !key_idx || !offs || (!msgs && offs[n] != offs[0])) return CESS_BLS_E_INVALID_ARG;
  if (c->nkeys == 0) return CESS_BLS_E_INVALID_ARG;
  // an out-of-range key index would read past the table: reject it on the host
  for (size_t i = 0; i < n; i++)
    if (key_idx[i] >= c->nkeys) return CESS_BLS_E_INVALID_ARG;
  HIPCHK(hipSetDevice(c->device));
  hipStream_t s = c->stream;
  std::vector<uint64_t> rebased, words;
  for (size_t off = 0; off < n; off += c->cap) {
    uint64_t m = std::min<uint64_t>(c->cap, n - off);
    uint64_t mb0 = offs[off], mb1 = offs[off + m];
    if (mb1 < mb0) return CESS_BLS_E_INVALID_ARG;
    rebased.resize(m + 1);
    for (uint64_t j = 0; j <= m; j++) {
      if (j && offs[off + j] < offs[off + j - 1]) return CESS_BLS_E_INVALID_ARG;
      rebased[j] = offs[off + j] - mb0;
    }
    int r = c->in_sigs.ensure(m * 48) | c->in_idx.ensure(m * 4) | c->in_msgs.ensure(std::max<uint64_t>(mb1 - mb0, 1)) |
            c->in_offs.ensure((m + 1) * 8);
    if (r) return CESS_BLS_E_OOM;
    HIPCHK(hipMemcpyAsync(c->in_sigs.p, sigs + 48 * off, m * 48, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(c->in_idx.p, key_idx + off, m * 4, hipMemcpyHostToDevice, s));
    if (mb1 > mb0) HIPCHK(hipMemcpyAsync(c->in_msgs.p, msgs + mb0, mb1 - mb0, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(c->in_offs.p, rebased.data(), (m + 1) * 8, hipMemcpyHostToDevice, s));
    r = run_chunk_keyed(c, s, m, c->in_sigs.as<uint8_t>(), c->in_idx.as<uint32_t>(), c->in_msgs.as<uint8_t>(),
                        c->in_offs.as<uint64_t>(), c->code.as<uint8_t>(), c->bitmap.as<uint64_t>());
    if (r) return r;
    if (codes_out) HIPCHK(hipMemcpyAsync(codes_out + off, c->code.p, m, hipMemcpyDeviceToHost, s));
    uint64_t nw = (m + 63) / 64;
    words.resize(nw);
    HIPCHK(hipMemcpyAsync(words.data(), c->bitmap.p, nw * 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (bitmap_out) memcpy(bitmap_out + off / 64, words.data(), nw * 8);
    r = collect_profile(c, s);
    if (r) return r;
  }
  return CESS_BLS_OK;
}

// generator-side batches -----------------------------------------------------
static int gen_batch(cess_bls_ctx* c, int kind, size_t n, const uint8_t* sks, const uint8_t* msgs, const uint64_t* offs,
                     uint8_t* out) {
  if (!c || !out) return CESS_BLS_E_INVALID_ARG;
  if (n == 0) return CESS_BLS_OK;
  HIPCHK(hipSetDevice(c->device));
  hipStream_t s = c->stream;
  const size_t ob = kind == 0 ? 96 : 48;
  std::vector<uint64_t> rebased;
  for (size_t off = 0; off < n; off += c->cap) {
    uint64_t m = std::min<uint64_t>(c->cap, n - off);
    int r = c->out_bytes.ensure(m * ob);
    if (kind != 2) r |= c->in_sks.ensure(m * 32);
    if (r) return CESS_BLS_E_OOM;
    if (kind != 2) HIPCHK(hipMemcpyAsync(c->in_sks.p, sks + 32 * off, m * 32, hipMemcpyHostToDevice, s));
    if (kind != 0) {
      uint64_t mb0 = offs[off], mb1 = offs[off + m];
      rebased.resize(m + 1);
      for (uint64_t j = 0; j <= m; j++) rebased[j] = offs[off + j] - mb0;
      r = c->in_msgs.ensure(std::max<uint64_t>(mb1 - mb0, 1)) | c->in_offs.ensure((m + 1) * 8);
      if (r) return CESS_BLS_E_OOM;
      if (mb1 > mb0) HIPCHK(hipMemcpyAsync(c->in_msgs.p, msgs + mb0, mb1 - mb0, hipMemcpyHostToDevice, s));
      HIPCHK(hipMemcpyAsync(c->in_offs.p, rebased.data(), (m + 1) * 8, hipMemcpyHostToDevice, s));
    }
    unsigned g = grid_for(m);
    if (kind == 0)
      hipLaunchKernelGGL(k_keygen, dim3(g), dim3(kBlock), 0, s, m, c->in_sks.as<uint8_t>(), c->out_bytes.as<uint8_t>());
    else if (kind == 1)
      hipLaunchKernelGGL(k_sign, dim3(g), dim3(kBlock), 0, s, m, c->in_sks.as<uint8_t>(), c->in_msgs.as<uint8_t>(),
                         c->in_offs.as<uint64_t>(), c->out_bytes.as<uint8_t>());
    else
      hipLaunchKernelGGL(k_hash_out, dim3(g), dim3(kBlock), 0, s, m, c->in_msgs.as<uint8_t>(), c->in_offs.as<uint64_t>(),
                         c->out_bytes.as<uint8_t>());
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(out + ob * off, c->out_bytes.p, m * ob, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
  }
  return CESS_BLS_OK;
}

extern "C" int cess_bls_public_key_batch(cess_bls_ctx* c, size_t n, const uint8_t* sks, uint8_t* pks_out) {
  if (!sks && n) return CESS_BLS_E_INVALID_ARG;
  return gen_batch(c, 0, n, sks, nullptr, nullptr, pks_out);
}
extern "C" int cess_bls_sign_batch(cess_bls_ctx* c, size_t n, const uint8_t* sks, const uint8_t* msgs,
                                   const uint64_t* offs, uint8_t* sigs_out) {
  if ((!sks || !offs) && n) return CESS_BLS_E_INVALID_ARG;
  return gen_batch(c, 1, n, sks, msgs, offs, sigs_out);
}
extern "C" int cess_bls_hash_to_g1_batch(cess_bls_ctx* c, size_t n, const uint8_t* msgs, const uint64_t* offs,
                                         uint8_t* out48) {
  if (!offs && n) return CESS_BLS_E_INVALID_ARG;
  return gen_batch(c, 2, n, nullptr, msgs, offs, out48);
}

extern "C" int cess_bls_stage_times(cess_bls_ctx* c, const char** names, double* ms, int max, int reset) {
  if (!c) return CESS_BLS_E_INVALID_ARG;
  int k = std::min(max, (int)ST_N);
  for (int i = 0; i < k; i++) {
    if (names) names[i] = kStageNames[i];
    if (ms) ms[i] = c->stage_ms[i];
  }
  if (reset)
    for (int i = 0; i < ST_N; i++) c->stage_ms[i] = 0;
  return ST_N;
}

// ---------------------------------------------------------------------------
// RLC batch mode (north_star).  One random linear
// combination per (sub)batch; on failure the batch is bisected down to leaves
// of kRlcLeaf records, which are verified per signature, so the final codes are
// those of cess_bls_verify_batch (up to the 2^-127 soundness error).
// ---------------------------------------------------------------------------
static constexpr uint64_t kRlcLeaf = 2048;   // records verified per signature
static constexpr uint64_t kRlcFan = 16;     // bisection fan-out per level

// Segmented sums: out[s] (stride out_stride) = sum of in[perm[off_s + j]], j < cnt_s.
// Two passes of k_g1_sum_segs (B partial sums per segment, then one).
static int rlc_sums(cess_bls_ctx* c, RlcState& R, hipStream_t s, const std::vector<uint64_t>& off,
                    const std::vector<uint64_t>& cnt, const uint32_t* in, uint64_t in_stride, uint32_t* out,
                    uint64_t out_stride) {
  const uint64_t ns = off.size();
  uint64_t mx = 1;
  for (uint64_t v : cnt) mx = std::max(mx, v);
  const uint64_t B = std::max<uint64_t>(1, std::min<uint64_t>(std::max<uint64_t>(1, 1024 / ns), (mx + 255) / 256));
  std::vector<uint64_t> h(4 * ns);
  for (uint64_t q = 0; q < ns; q++) h[q] = off[q], h[ns + q] = cnt[q], h[2 * ns + q] = q * B, h[3 * ns + q] = B;
  if (R.seg.ensure(h.size() * 8) || R.part.ensure(ns * B * 36 * 4)) return CESS_BLS_E_OOM;
  HIPCHK(hipMemcpyAsync(R.seg.p, h.data(), h.size() * 8, hipMemcpyHostToDevice, s));
  const uint64_t* d = R.seg.as<uint64_t>();
  hipLaunchKernelGGL(k_g1_sum_segs, dim3((unsigned)B, (unsigned)ns), dim3(256), 0, s, d, d + ns,
                     (const uint32_t*)R.d_perm.as<uint32_t>(), in, in_stride, R.part.as<uint32_t>(), ns * B);
  hipLaunchKernelGGL(k_g1_sum_segs, dim3(1, (unsigned)ns), dim3(256), 0, s, d + 2 * ns, d + 3 * ns,
                     (const uint32_t*)nullptr, (const uint32_t*)R.part.as<uint32_t>(), ns * B, out, out_stride);
  HIPCHK(hipGetLastError());
  // the host vector h must outlive the async copy
  HIPCHK(hipStreamSynchronize(s));
  return CESS_BLS_OK;
}

// RLC checks of NR perm-position ranges in one batch: ok[r] = the product of
// range r's K+1 pairings is 1.  gt_out (optional, NR == 1): its Gt value.
static int rlc_check_multi(cess_bls_ctx* c, RlcState& R, const std::vector<std::pair<uint64_t, uint64_t>>& rg,
                           std::vector<uint8_t>& ok, uint8_t* gt_out) {
  hipStream_t s = c->stream;
  const uint32_t K = R.K, NR = (uint32_t)rg.size(), M = NR * K;
  R.checks += NR;
  std::vector<uint64_t> so(NR), sc(NR), qo(M), qc(M);
  for (uint32_t r = 0; r < NR; r++) {
    const uint64_t a = rg[r].first, b = rg[r].second;
    so[r] = a, sc[r] = b - a;
    for (uint32_t g = 0; g < K; g++) {
      const uint64_t lo = std::max(a, R.gbeg[g]), hi = std::min(b, R.gbeg[g + 1]);
      qo[r * K + g] = lo, qc[r * K + g] = hi > lo ? hi - lo : 0;
    }
  }
  int r = 0;
  r |= R.S.ensure((uint64_t)NR * 36 * 4) | R.Qs.ensure((uint64_t)M * 36 * 4);
  r |= R.rec_code.ensure(M) | R.rec_inf.ensure(M) | R.rec_sig.ensure((uint64_t)M * CESS_W_G1 * 4);
  r |= R.rec_h.ensure((uint64_t)M * CESS_W_G1 * 4) | R.rec_f.ensure((uint64_t)M * CESS_W_FP12 * 4) |
       R.rec_f2.ensure((uint64_t)M * CESS_W_FP12 * 4);
  r |= R.acc.ensure((uint64_t)NR * CESS_W_FP12 * 4) | R.slots.ensure((uint64_t)NR * CESS_W_FP12 * 4 * CESS_FE_SLOTS);
  r |= R.fin_code.ensure(NR) | R.fin_bm.ensure(((NR + 63) / 64) * 8) | R.gt.ensure((uint64_t)NR * 576);
  if (NR > 1) r |= R.rec_coeffs.ensure((uint64_t)M * CESS_W_COEFFS * 4);
  if (r) return CESS_BLS_E_OOM;
  r = rlc_sums(c, R, s, so, sc, R.P.as<uint32_t>(), R.n, R.S.as<uint32_t>(), NR);
  if (r) return r;
  r = rlc_sums(c, R, s, qo, qc, R.Q.as<uint32_t>(), R.n, R.Qs.as<uint32_t>(), M);
  if (r) return r;
  const uint4* coeffs = R.pk_coeffs.as<uint4>();
  if (NR > 1) {
    const uint64_t rows = CESS_W_COEFFS / 4, tot = rows * M;
    hipLaunchKernelGGL(k_rep_rows, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, (uint32_t)rows, NR, K,
                       coeffs, R.rec_coeffs.as<uint4>());
    coeffs = R.rec_coeffs.as<uint4>();
  }
  hipLaunchKernelGGL(k_rlc_pairs_multi, dim3((M + 63) / 64), dim3(64), 0, s, NR, K, (const uint32_t*)R.S.as<uint32_t>(),
                     (const uint32_t*)R.Qs.as<uint32_t>(), (const uint8_t*)R.pk_usable.as<uint8_t>(),
                     R.rec_code.as<uint8_t>(), R.rec_inf.as<uint8_t>(), R.rec_sig.as<uint32_t>(), R.rec_h.as<uint32_t>());
  hipLaunchKernelGGL(k_miller, dim3((M + kBlock - 1) / kBlock), dim3(kBlock), 0, s, (uint64_t)M,
                     (const uint8_t*)R.rec_code.as<uint8_t>(), (const uint8_t*)R.rec_inf.as<uint8_t>(),
                     (const uint32_t*)R.rec_sig.as<uint32_t>(), (const uint32_t*)R.rec_h.as<uint32_t>(),
                     (const uint32_t*)c->neg_g2.as<uint32_t>(), coeffs, R.rec_f.as<uint4>(), R.rec_f2.as<uint4>(),
                     (uint64_t)M, (const uint32_t*)nullptr, (uint64_t)M);
  hipLaunchKernelGGL(k_fp12_prod_multi, dim3((NR + 63) / 64), dim3(64), 0, s, NR, K, (const uint4*)R.rec_f.as<uint4>(),
                     R.acc.as<uint4>());
  HIPCHK(hipMemsetAsync(R.fin_code.p, 0, NR, s));
  hipLaunchKernelGGL(k_final, dim3((NR + kBlock - 1) / kBlock), dim3(kBlock), 0, s, (uint64_t)NR,
                     R.fin_code.as<uint8_t>(), R.acc.as<uint4>(), R.slots.as<uint4>(), R.fin_bm.as<uint64_t>(),
                     gt_out ? R.gt.as<uint8_t>() : (uint8_t*)nullptr, (uint64_t)NR);
  HIPCHK(hipGetLastError());
  ok.assign(NR, 0);
  std::vector<uint8_t> codes(NR);
  HIPCHK(hipMemcpyAsync(codes.data(), R.fin_code.p, NR, hipMemcpyDeviceToHost, s));
  if (gt_out) HIPCHK(hipMemcpyAsync(gt_out, R.gt.p, 576, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  for (uint32_t q = 0; q < NR; q++) ok[q] = codes[q] == CODE_OK;
  return CESS_BLS_OK;
}

extern "C" int cess_bls_rlc_begin(cess_bls_ctx* c, size_t n, const uint8_t* sigs, const uint8_t* pks,
                                  const uint8_t* msgs, const uint64_t* offs, const uint8_t* seed32, uint8_t* gt_out) {
  if (!c || !seed32 || (n && (!sigs || !pks || !offs || (!msgs && offs[n] != offs[0])))) return CESS_BLS_E_INVALID_ARG;
  if (n >= (1ull << 32)) return CESS_BLS_E_INVALID_ARG;
  HIPCHK(hipSetDevice(c->device));
  if (!c->rlc) c->rlc = new RlcState();
  RlcState& R = *c->rlc;
  R.n = n, R.sigs = sigs, R.pks = pks, R.msgs = msgs, R.offs = offs;
  R.checks = R.leaves = R.leaf_sigs = 0;
  R.codes.assign(n, 0);
  R.local_ok = true;
  if (n == 0) {
    if (gt_out) {   // the empty product: Gt one
      memset(gt_out, 0, 576);
      gt_out[47] = 1;
    }
    R.K = 0;
    return CESS_BLS_OK;
  }
  hipStream_t s = c->stream;
  // 1. key groups (dedup of the 96-byte encodings; open addressing on a
  //    64-bit hash, full compare) and a counting sort by group
  std::vector<uint32_t> grp(n);
  std::vector<uint64_t> first;
  {
    auto khash = [](const uint8_t* k) {
      uint64_t h = 0x9E3779B97F4A7C15ull;
      for (int q = 0; q < 96; q += 8) {
        uint64_t w;
        memcpy(&w, k + q, 8);
        h = (h ^ w) * 0xff51afd7ed558ccdull;
        h ^= h >> 29;
      }
      return h;
    };
    std::vector<uint32_t> slot(64, 0);   // group id + 1; 0 = empty
    uint64_t mask = 63;
    for (uint64_t i = 0; i < n; i++) {
      const uint8_t* k = pks + 96 * i;
      uint64_t h = khash(k) & mask;
      while (slot[h] && memcmp(pks + 96 * first[slot[h] - 1], k, 96) != 0) h = (h + 1) & mask;
      if (!slot[h]) {
        first.push_back(i);
        slot[h] = (uint32_t)first.size();
        if (2 * first.size() > mask) {   // grow and rehash
          std::vector<uint32_t> ns(2 * (mask + 1), 0);
          const uint64_t nm = 2 * (mask + 1) - 1;
          for (uint32_t g = 0; g < first.size(); g++) {
            uint64_t q = khash(pks + 96 * first[g]) & nm;
            while (ns[q]) q = (q + 1) & nm;
            ns[q] = g + 1;
          }
          slot.swap(ns);
          mask = nm;
        }
        grp[i] = (uint32_t)first.size() - 1;
      } else {
        grp[i] = slot[h] - 1;
      }
    }
  }
  const uint32_t K = R.K = (uint32_t)first.size();
  R.gbeg.assign(K + 1, 0);
  for (uint64_t i = 0; i < n; i++) R.gbeg[grp[i] + 1]++;
  for (uint32_t g = 0; g < K; g++) R.gbeg[g + 1] += R.gbeg[g];
  R.perm.resize(n);
  {
    std::vector<uint64_t> pos(R.gbeg.begin(), R.gbeg.end() - 1);
    for (uint64_t i = 0; i < n; i++) R.perm[pos[grp[i]]++] = (uint32_t)i;
  }
  // 2. device buffers
  int r = 0;
  r |= R.P.ensure(n * 36 * 4) | R.Q.ensure(n * 36 * 4) | R.d_perm.ensure(n * 4) | R.d_seed.ensure(32);
  r |= R.pk_in.ensure((uint64_t)K * 96);
  r |= R.pk_code.ensure(K) | R.pk_inf.ensure(K) | R.pk_aff.ensure((uint64_t)K * CESS_W_G2 * 4);
  r |= R.pk_coeffs.ensure((uint64_t)K * CESS_W_COEFFS * 4) | R.pk_usable.ensure(K);
  if (r) return CESS_BLS_E_OOM;
  {
    uint32_t sw[8];
    for (int w = 0; w < 8; w++)
      sw[w] = ((uint32_t)seed32[4 * w] << 24) | ((uint32_t)seed32[4 * w + 1] << 16) | ((uint32_t)seed32[4 * w + 2] << 8) |
              seed32[4 * w + 3];
    HIPCHK(hipMemcpyAsync(R.d_seed.p, sw, 32, hipMemcpyHostToDevice, s));
  }
  HIPCHK(hipMemcpyAsync(R.d_perm.p, R.perm.data(), n * 4, hipMemcpyHostToDevice, s));
  // 3. distinct keys: decode (G2Affine::from_compressed, src/lib.rs:74) + G2Prepared (:88), once per key
  std::vector<uint8_t> kbytes((uint64_t)K * 96), pkc(K), pki(K), usable(K);
  for (uint32_t g = 0; g < K; g++) memcpy(&kbytes[96 * (uint64_t)g], pks + 96 * first[g], 96);
  HIPCHK(hipMemcpyAsync(R.pk_in.p, kbytes.data(), kbytes.size(), hipMemcpyHostToDevice, s));
  HIPCHK(hipMemsetAsync(R.pk_code.p, 0, K, s));
  HIPCHK(hipMemsetAsync(R.pk_inf.p, 0, K, s));
  hipLaunchKernelGGL(k_decode_pk, dim3(grid_for(K)), dim3(kBlock), 0, s, (uint64_t)K, R.pk_in.as<uint8_t>(),
                     (const uint8_t*)nullptr, R.pk_code.as<uint8_t>(), R.pk_inf.as<uint8_t>(), R.pk_aff.as<uint32_t>(),
                     (uint64_t)K);
  hipLaunchKernelGGL(k_prepare, dim3(grid_for(K)), dim3(kBlock), 0, s, (uint64_t)K,
                     (const uint32_t*)R.pk_aff.as<uint32_t>(), R.pk_coeffs.as<uint4>(), (uint64_t)K);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(pkc.data(), R.pk_code.p, K, hipMemcpyDeviceToHost, s));
  HIPCHK(hipMemcpyAsync(pki.data(), R.pk_inf.p, K, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  for (uint32_t g = 0; g < K; g++) usable[g] = pkc[g] == 0 && !(pki[g] & INF_PK);
  HIPCHK(hipMemcpyAsync(R.pk_usable.p, usable.data(), K, hipMemcpyHostToDevice, s));
  // 4. per chunk: decode sig (src/lib.rs:144), key codes in reference precedence
  //    (signature first, :244-245), hash_to_g1 (:25-31), P_i = r_i sig_i, Q_i = r_i H_i
  std::vector<uint8_t> hc, hi;
  std::vector<uint64_t> rebased;
  for (uint64_t off = 0; off < n; off += c->cap) {
    const uint64_t m = std::min<uint64_t>(c->cap, n - off);
    const uint64_t mb0 = offs[off], mb1 = offs[off + m];
    rebased.resize(m + 1);
    for (uint64_t j = 0; j <= m; j++) {
      if (j && offs[off + j] < offs[off + j - 1]) return CESS_BLS_E_INVALID_ARG;
      rebased[j] = offs[off + j] - mb0;
    }
    r = c->in_sigs.ensure(m * 48) | c->in_msgs.ensure(std::max<uint64_t>(mb1 - mb0, 1)) | c->in_offs.ensure((m + 1) * 8);
    if (r) return CESS_BLS_E_OOM;
    HIPCHK(hipMemcpyAsync(c->in_sigs.p, sigs + 48 * off, m * 48, hipMemcpyHostToDevice, s));
    if (mb1 > mb0) HIPCHK(hipMemcpyAsync(c->in_msgs.p, msgs + mb0, mb1 - mb0, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(c->in_offs.p, rebased.data(), (m + 1) * 8, hipMemcpyHostToDevice, s));
    const unsigned g = grid_for(m);
    hipLaunchKernelGGL(k_decode_sig, dim3(g), dim3(kBlock), 0, s, m, c->in_sigs.as<uint8_t>(), (const uint8_t*)nullptr,
                       c->code.as<uint8_t>(), c->inf.as<uint8_t>(), c->sig_aff.as<uint32_t>(), c->cap);
    HIPCHK(hipGetLastError());
    hc.resize(m);
    hi.resize(m);
    HIPCHK(hipMemcpyAsync(hc.data(), c->code.p, m, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(hi.data(), c->inf.p, m, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    for (uint64_t j = 0; j < m; j++) {
      if (hc[j] != 0) continue;
      const uint32_t gg = grp[off + j];
      if (pkc[gg] != 0) hc[j] = pkc[gg];
      else if (pki[gg] & INF_PK) hi[j] |= INF_PK;
    }
    memcpy(&R.codes[off], hc.data(), m);
    HIPCHK(hipMemcpyAsync(c->code.p, hc.data(), m, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(c->inf.p, hi.data(), m, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_hash, dim3(g), dim3(kBlock), 0, s, m, c->in_msgs.as<uint8_t>(), c->in_offs.as<uint64_t>(),
                       (const uint8_t*)c->code.as<uint8_t>(), c->h_aff.as<uint32_t>(), c->cap);
    hipLaunchKernelGGL(k_rlc_scale, dim3(g), dim3(kBlock), 0, s, m, (const uint8_t*)c->code.as<uint8_t>(),
                       (const uint8_t*)c->inf.as<uint8_t>(), (const uint32_t*)c->sig_aff.as<uint32_t>(),
                       (const uint32_t*)c->h_aff.as<uint32_t>(), (const uint32_t*)R.d_seed.as<uint32_t>(), off,
                       R.P.as<uint32_t>() + off, R.Q.as<uint32_t>() + off, c->cap, n);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(s));   // hc/hi are reused by the next chunk
  }
  // 5. the batch check (this shard's Gt partial)
  std::vector<uint8_t> ok;
  r = rlc_check_multi(c, R, {{0, n}}, ok, gt_out);
  if (r) return r;
  R.local_ok = ok[0] != 0;
  return CESS_BLS_OK;
}

extern "C" int cess_bls_gt_product_is_one(cess_bls_ctx* c, size_t m, const uint8_t* gts, int* is_one) {
  if (!c || !is_one || (m && !gts)) return CESS_BLS_E_INVALID_ARG;
  HIPCHK(hipSetDevice(c->device));
  if (!c->rlc) c->rlc = new RlcState();
  RlcState& R = *c->rlc;
  if (m == 0) {
    *is_one = 1;
    return CESS_BLS_OK;
  }
  hipStream_t s = c->stream;
  if (R.gts.ensure(m * 576) | R.tmp.ensure(2 * CESS_W_FP12 * 4) | R.fin_code.ensure(1)) return CESS_BLS_E_OOM;
  HIPCHK(hipMemcpyAsync(R.gts.p, gts, m * 576, hipMemcpyHostToDevice, s));
  hipLaunchKernelGGL(k_gt_prod, dim3(1), dim3(64), 0, s, (uint32_t)m, (const uint8_t*)R.gts.as<uint8_t>(),
                     R.tmp.as<uint4>(), R.fin_code.as<uint8_t>());
  HIPCHK(hipGetLastError());
  uint8_t code = 0xff;
  HIPCHK(hipMemcpyAsync(&code, R.fin_code.p, 1, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  *is_one = code == CODE_OK;
  return CESS_BLS_OK;
}

extern "C" int cess_bls_rlc_finish(cess_bls_ctx* c, int global_ok, uint8_t* codes_out, uint64_t* bitmap_out,
                                   uint64_t* stats4) {
  if (!c || !c->rlc) return CESS_BLS_E_INVALID_ARG;
  RlcState& R = *c->rlc;
  const uint64_t n = R.n;
  std::vector<uint8_t>& codes = R.codes;
  if (!global_ok && !R.local_ok) {
    // batched bisection over perm positions: every failing range is split
    // into up to kRlcFan parts, all parts of a level are checked in one batch;
    // ranges of <= kRlcLeaf records are verified per signature (exact codes)
    std::vector<std::pair<uint64_t, uint64_t>> level = {{0, n}}, parts, leaves;
    std::vector<uint8_t> ok;
    while (!level.empty()) {
      parts.clear();
      for (auto& w : level) {
        const uint64_t len = w.second - w.first;
        if (len <= kRlcLeaf) {
          leaves.push_back(w);
          continue;
        }
        const uint64_t fan = std::min<uint64_t>(kRlcFan, (len + kRlcLeaf - 1) / kRlcLeaf);
        for (uint64_t q = 0; q < fan; q++)
          parts.push_back({w.first + len * q / fan, w.first + len * (q + 1) / fan});
      }
      level.clear();
      if (!parts.empty()) {
        int r = rlc_check_multi(c, R, parts, ok, nullptr);
        if (r) return r;
        for (size_t q = 0; q < parts.size(); q++)
          if (!ok[q]) level.push_back(parts[q]);
      }
    }
    // leaves: one per-signature batch over all their candidate records
    std::vector<uint64_t> li, lo = {0};
    std::vector<uint8_t> ls, lp, lm, lc;
    for (auto& w : leaves) {
      for (uint64_t j = w.first; j < w.second; j++)
        if (codes[R.perm[j]] == 0) li.push_back(R.perm[j]);
      R.leaves++;
    }
    const uint64_t m = li.size();
    if (m) {
      ls.resize(m * 48);
      lp.resize(m * 96);
      for (uint64_t q = 0; q < m; q++) {
        const uint64_t i = li[q];
        memcpy(&ls[48 * q], R.sigs + 48 * i, 48);
        memcpy(&lp[96 * q], R.pks + 96 * i, 96);
        lm.insert(lm.end(), R.msgs + R.offs[i], R.msgs + R.offs[i + 1]);
        lo.push_back(lm.size());
      }
      lc.resize(m);
      int r = verify_host(c, m, ls.data(), lp.data(), lm.empty() ? nullptr : lm.data(), lo.data(), nullptr, lc.data(),
                          nullptr, nullptr);
      if (r) return r;
      for (uint64_t q = 0; q < m; q++) codes[li[q]] = lc[q];
      R.leaf_sigs += m;
    }
  }
  if (codes_out) memcpy(codes_out, codes.data(), n);
  if (bitmap_out) {
    for (uint64_t w = 0; w < (n + 63) / 64; w++) bitmap_out[w] = 0;
    for (uint64_t i = 0; i < n; i++)
      if (codes[i] == 0) bitmap_out[i >> 6] |= 1ull << (i & 63);
  }
  if (stats4) {
    stats4[0] = R.checks;
    stats4[1] = R.leaves;
    stats4[2] = R.leaf_sigs;
    stats4[3] = R.K;
  }
  return CESS_BLS_OK;
}

extern "C" int cess_bls_verify_batch_rlc(cess_bls_ctx* c, size_t n, const uint8_t* sigs, const uint8_t* pks,
                                         const uint8_t* msgs, const uint64_t* msg_offsets, const uint8_t* seed32,
                                         uint8_t* codes_out, uint64_t* bitmap_out, uint64_t* stats4) {
  int r = cess_bls_rlc_begin(c, n, sigs, pks, msgs, msg_offsets, seed32, nullptr);
  if (r) return r;
  return cess_bls_rlc_finish(c, c->rlc->local_ok, codes_out, bitmap_out, stats4);
}
