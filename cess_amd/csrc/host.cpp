// Host runtime behind include/cess_bls.h: one context per GPU, a HIP stream,
// device stage buffers sized for one launch chunk, and the constant
// G2PREPARED_NEG_G table (reference src/lib.rs:19-21) built once on the device.
// (RLC mode: host_rlc.cpp; RCCL communicator, sharded batches and multi-device
// contexts: host_multi.cpp.)
//
// There is no CPU compute path: every verdict is produced by the gfx950 kernels.
// Without a usable HIP device, cess_bls_ctx_create fails with CESS_BLS_E_NO_DEVICE.
#include "host.hpp"

#include <stdlib.h>
#include <string.h>

#include "bls/consts.hpp"

using namespace cess_host;

namespace {
const char* kStageNames[ST_N] = {"k_decode_sig", "k_decode_pk",    "k_hash",       "k_prepare", "k_miller",
                                 "k_final",      "k_rsa_classify", "k_rsa_verify", "k_group",  "k_sign"};
}

extern "C" const char* cess_bls_version(void) { return "cess_amd-bls 0.2 (gfx950)"; }

extern "C" int cess_bls_device_count(void) {
  int n = 0;
  return hipGetDeviceCount(&n) == hipSuccess && n > 0 ? n : 0;
}

extern "C" const char* cess_bls_status_string(int s) {
  switch (s) {
    case CESS_BLS_OK: return "ok";
    case CESS_BLS_E_INVALID_ARG: return "invalid argument";
    case CESS_BLS_E_NO_DEVICE: return "no HIP device (the verifier has no CPU fallback)";
    case CESS_BLS_E_HIP: return "HIP runtime error";
    case CESS_BLS_E_OOM: return "device out of memory";
    case CESS_BLS_E_RCCL: return "RCCL error";
    case CESS_BLS_E_BUSY: return "context in use by another thread";
    case CESS_BLS_E_BAD_KEY: return "public key does not deserialize (verify_bls would panic)";
    case CESS_BLS_E_BAD_SIG: return "signature does not deserialize (verify_bls would panic)";
    case CESS_BLS_E_NO_COMM: return "no communicator (cess_bls_comm_init / cess_bls_comm_init_shm)";
    case CESS_BLS_E_COMM: return "communicator failed (peer timeout, or the communicator was aborted)";
    case CESS_RSA_E_UNSUPPORTED: return "RSA key not supported on the GPU (> 2048-bit, even modulus or non-NULL parameters): the caller's CPU path decides";
  }
  return "unknown status";
}

namespace cess_host {

int order_begin(cess_bls_ctx* c, hipStream_t s) {
  if (c->pending && c->last_stream != s) HIPCHK(hipStreamWaitEvent(s, c->done_ev, 0));
  return CESS_BLS_OK;
}

int order_end(cess_bls_ctx* c, hipStream_t s) {
  HIPCHK(hipEventRecord(c->done_ev, s));
  c->last_stream = s;
  c->pending = true;
  return CESS_BLS_OK;
}

void bitmap_from_codes(const uint8_t* codes, uint64_t n, uint64_t* words) {
  for (uint64_t w = 0; w < (n + 63) / 64; w++) words[w] = 0;
  for (uint64_t i = 0; i < n; i++)
    if (codes[i] == CODE_OK) words[i >> 6] |= 1ull << (i & 63);
}

void shard_of(uint64_t n, int nranks, int rank, uint64_t* begin, uint64_t* end, uint64_t* wpr) {
  const uint64_t words = (n + 63) / 64;
  const uint64_t per = nranks > 0 ? (words + nranks - 1) / nranks : 0;
  const uint64_t b = std::min<uint64_t>(n, (uint64_t)rank * per * 64);
  const uint64_t e = std::min<uint64_t>(n, ((uint64_t)rank + 1) * per * 64);
  if (begin) *begin = b;
  if (end) *end = e;
  if (wpr) *wpr = per;
}

}  // namespace cess_host

static int alloc_stage(cess_bls_ctx* c) {
  const uint64_t n = c->cap, q = c->qcap;
  int r = CESS_BLS_OK;
  r |= c->pre.ensure(n);
  r |= c->code.ensure(n);
  r |= c->bitmap.ensure((n / 64 + 1) * 8);
  r |= c->fval.ensure(q * CESS_W_FP12 * 4);
  r |= c->fe_slots.ensure(q * CESS_W_FP12 * 4 * CESS_FE_SLOTS);
  for (int k = 0; k < (q < n ? 2 : 1); k++) {
    r |= c->slot[k].inf.ensure(q);
    r |= c->slot[k].sig_aff.ensure(q * CESS_W_G1 * 4);
    r |= c->slot[k].h_aff.ensure(q * CESS_W_G1 * 4);
  }
  return r ? CESS_BLS_E_OOM : CESS_BLS_OK;
}

// records per kernel launch: the whole chunk by default.  Pipelining parts of
// 2^17-2^19 records (light kernels of part i+1 beside k_miller of part i) was
// measured SLOWER on MI355X (1.970 M sigs/s unpipelined vs 1.914 / 1.873 /
// 1.879 M at 512K / 256K / 128K parts, profiles/r02c_sweep_launch_records.txt:
// k_miller slows from 187 to 263 ms per 1 M when co-resident waves share its
// SIMDs; re-measured with the round-5 kernels: 2.74 M unpipelined vs 2.65 /
// 2.51 M at 512K / 256K parts, k_miller 149 -> 200 ms,
// profiles/round5_al_sweep_launch_records.txt), so the mechanism stays
// available via CESS_BLS_LAUNCH_RECORDS only.
static uint64_t launch_records(uint64_t cap) {
  uint64_t q = cap;
  if (const char* e = getenv("CESS_BLS_LAUNCH_RECORDS")) q = strtoull(e, nullptr, 10);
  q = std::max<uint64_t>(256, q & ~255ull);
  return std::min(cap, q);
}

// Batches of at most this many records run the lane-group path (k_group: one
// signature per wave): below it the one-lane-per-signature
// pipeline costs one lane's latency through six kernels whatever the batch
// size.  Env CESS_BLS_SMALL_BATCH (0 disables).
static uint64_t small_records() {
  // measured crossover: with the round-6 lane-pair heavy kernels the pipeline
  // takes 17.0-17.4 ms from 4,096 to 5,632 records against k_group's 13.7 /
  // 16.2 / 18.7 ms at 4,096 / 5,120 / 5,632 (profiles/round6_ap_latency.txt,
  // round6_aq_latency.txt; 8,192 in rounds 3-5, profiles/round3_*_latency.txt)
  uint64_t v = 5120;
  if (const char* e = getenv("CESS_BLS_SMALL_BATCH")) v = strtoull(e, nullptr, 10);
  return v;
}

// The Miller loop kernel: k_miller2 (default: a lane pair per signature,
// 256-thread blocks of 128 signatures, two waves per SIMD; bls/pair.hpp) or
// k_miller (one lane per signature, one wave per SIMD), env CESS_BLS_MILLER =
// lane.  Both take the same arguments and write the same fval rows; k_miller2
// runs config[1]'s Miller loop in 129.8-130.0 ms per 1 M against 149.5-149.7
// (same box, profiles/round6_c_sweep_miller_pair.txt).
typedef void (*MillerKernel)(uint64_t, const uint8_t*, const uint8_t*, const uint32_t*, const uint32_t*,
                             const uint32_t*, const uint4*, uint4*, uint4*, uint64_t, const uint32_t*, uint64_t,
                             const uint8_t*);
static bool miller_pair() {
  static const bool v = [] {
    const char* e = getenv("CESS_BLS_MILLER");
    return !(e && strcmp(e, "lane") == 0);
  }();
  return v;
}
static MillerKernel miller_kernel() { return miller_pair() ? k_miller2 : k_miller; }
// the lane-pair kernels: blocks of CESS_PAIR_THREADS / 2 signatures
constexpr uint64_t kPairSigs = CESS_PAIR_THREADS / 2;
// (covering whole 64-record bitmap words: k_final2 writes 32-bit halves, one per
// wave of 32 signatures, so both waves of a word must exist)
static unsigned pair_grid(uint64_t m) {
  const uint64_t m64 = (m + 63) & ~63ull;
  return (unsigned)((m64 + kPairSigs - 1) / kPairSigs);
}
static dim3 miller_grid(uint64_t m) { return dim3(miller_pair() ? pair_grid(m) : grid_for(m)); }
static dim3 miller_block() { return dim3(miller_pair() ? CESS_PAIR_THREADS : kBlock); }

// The final-exponentiation kernel: k_final2 (default: a lane pair per
// signature, the accumulator in LDS; bls/pair_fe.hpp) or k_final (one lane per
// signature, accumulators in HBM), env CESS_BLS_FINAL = lane.  Same arguments
// and outputs; k_final2 137.4-138.2 against 142.1 ms per 1 M on one box, ~99
// against ~332 KB/sig counted traffic (profiles/round6_e_sweep_final_pair.txt).
typedef void (*FinalKernel)(uint64_t, uint8_t*, uint4*, uint4*, uint64_t*, uint8_t*, uint64_t);
static bool final_pair() {
  static const bool v = [] {
    const char* e = getenv("CESS_BLS_FINAL");
    return !(e && strcmp(e, "lane") == 0);
  }();
  return v;
}
static FinalKernel final_kernel() { return final_pair() ? k_final2 : k_final; }
static dim3 final_grid(uint64_t m) { return dim3(final_pair() ? pair_grid(m) : grid_for(m)); }
static dim3 final_block() { return dim3(final_pair() ? CESS_PAIR_THREADS : kBlock); }

int cess_multi_create(const cess_bls_config* cfg, int ndev, cess_bls_ctx* c);   // host_multi.cpp

extern "C" int cess_bls_ctx_create(const cess_bls_config* cfg, cess_bls_ctx** out) {
  if (!out) return CESS_BLS_E_INVALID_ARG;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return CESS_BLS_E_NO_DEVICE;
  if (cfg && cfg->mode > CESS_BLS_MODE_RLC) return CESS_BLS_E_INVALID_ARG;
  if (cfg && cfg->n_devices > 1) {
    cess_bls_ctx* c = new cess_bls_ctx();
    int r = cess_multi_create(cfg, ndev, c);
    if (r != CESS_BLS_OK) {
      cess_bls_ctx_destroy(c);
      return r;
    }
    *out = c;
    return CESS_BLS_OK;
  }
  cess_bls_ctx* c = new cess_bls_ctx();
  c->device = (cfg && cfg->device >= 0) ? cfg->device : 0;
  if (c->device < 0 || c->device >= ndev) {
    delete c;
    return CESS_BLS_E_INVALID_ARG;
  }
  uint64_t cap = (cfg && cfg->max_batch) ? cfg->max_batch : (1ull << 20);
  c->cap = (cap + 63) & ~63ull;
  c->qcap = launch_records(c->cap);
  c->small = std::min(small_records(), c->qcap);
  c->flags = cfg ? cfg->flags : 0;
  c->mode = cfg ? cfg->mode : CESS_BLS_MODE_PER_SIG;
  bool ok = hipSetDevice(c->device) == hipSuccess &&
            hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) == hipSuccess &&
            hipStreamCreateWithFlags(&c->stream2, hipStreamNonBlocking) == hipSuccess &&
            hipStreamCreateWithFlags(&c->stream3, hipStreamNonBlocking) == hipSuccess &&
            hipEventCreateWithFlags(&c->done_ev, hipEventDisableTiming) == hipSuccess &&
            hipEventCreateWithFlags(&c->ev_start, hipEventDisableTiming) == hipSuccess;
  for (int k = 0; k < 2 && ok; k++)
    ok = hipEventCreateWithFlags(&c->ev_light[k], hipEventDisableTiming) == hipSuccess &&
         hipEventCreateWithFlags(&c->ev_mill[k], hipEventDisableTiming) == hipSuccess;
  if (!ok) {
    cess_bls_ctx_destroy(c);
    return CESS_BLS_E_HIP;
  }
  int r = alloc_stage(c);
  if (r == CESS_BLS_OK) r = c->neg_g2.ensure(CESS_W_COEFFS * 4);
  if (r != CESS_BLS_OK) {
    cess_bls_ctx_destroy(c);
    return r;
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
                     (uint64_t)1, (uint8_t*)nullptr, (const uint8_t*)nullptr);
  hipLaunchKernelGGL(k_norm_lines, dim3(1), dim3(128), 0, c->stream, c->neg_g2.as<uint4>());
  if (hipGetLastError() != hipSuccess || hipStreamSynchronize(c->stream) != hipSuccess) {
    cess_bls_ctx_destroy(c);
    return CESS_BLS_E_HIP;
  }
  *out = c;
  return CESS_BLS_OK;
}

extern "C" void cess_bls_ctx_destroy(cess_bls_ctx* c) {
  if (!c) return;
  for (cess_bls_ctx* s : c->subs) cess_bls_ctx_destroy(s);
  c->subs.clear();
  if (c->stream) {
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
  }
  if (c->stream2) (void)hipStreamSynchronize(c->stream2);
  if (c->stream3) (void)hipStreamSynchronize(c->stream3);
  delete c->xport;
  for (hipEvent_t e : c->evpool) (void)hipEventDestroy(e);
  for (hipEvent_t e : {c->done_ev, c->ev_start, c->ev_light[0], c->ev_light[1], c->ev_mill[0], c->ev_mill[1]})
    if (e) (void)hipEventDestroy(e);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  if (c->stream2) (void)hipStreamDestroy(c->stream2);
  if (c->stream3) (void)hipStreamDestroy(c->stream3);
  delete c->rlc;
  cess_rsa_state_free(c);
  delete c;
}

int cess_host::prof_begin(cess_bls_ctx* c, hipStream_t s, int stage, hipEvent_t* a) {
  (void)stage;
  *a = nullptr;
  if (!(c->flags & CESS_BLS_F_PROFILE)) return CESS_BLS_OK;
  if (c->evused == c->evpool.size()) {
    hipEvent_t e;
    HIPCHK(hipEventCreate(&e));
    c->evpool.push_back(e);
  }
  *a = c->evpool[c->evused++];
  HIPCHK(hipEventRecord(*a, s));
  return CESS_BLS_OK;
}

int cess_host::prof_end(cess_bls_ctx* c, hipStream_t s, int stage, hipEvent_t a) {
  if (!a) return CESS_BLS_OK;
  hipEvent_t b;
  int r = prof_begin(c, s, stage, &b);
  if (r) return r;
  c->prof.push_back({stage, a, b});
  return CESS_BLS_OK;
}

#define LAUNCH(stage, strm, ...)                        \
  do {                                                  \
    hipEvent_t pa_;                                     \
    int pr_ = prof_begin(c, strm, stage, &pa_);         \
    if (pr_) return pr_;                                \
    hipLaunchKernelGGL(__VA_ARGS__);                    \
    pr_ = prof_end(c, strm, stage, pa_);                \
    if (pr_) return pr_;                                \
  } while (0)

// The pipeline over one chunk of n <= cap records, in parts of <= qcap.
// light(S, q, off, m, strm) enqueues the part's decode/hash(/prepare) kernels
// into stage slot S on strm; heavy(S, q, off, m) its Miller loop and final
// exponentiation on the launch stream s.  One part runs on s alone; with
// several, the light kernels run one part ahead on stream2 (slot = part % 2).
template <class Light, class Heavy>
static int pipeline(cess_bls_ctx* c, hipStream_t s, uint64_t n, Light&& light, Heavy&& heavy) {
  const uint64_t q = c->qcap;
  if (n <= q) {
    int r = light(c->slot[0], q, (uint64_t)0, n, s);
    if (r) return r;
    return heavy(c->slot[0], q, (uint64_t)0, n);
  }
  hipStream_t s2 = c->stream2;
  HIPCHK(hipEventRecord(c->ev_start, s));
  HIPCHK(hipStreamWaitEvent(s2, c->ev_start, 0));
  for (uint64_t off = 0, part = 0; off < n; off += q, part++) {
    const uint64_t m = std::min(q, n - off);
    const int k = (int)(part & 1);
    StageSlot& S = c->slot[k];
    if (part >= 2) HIPCHK(hipStreamWaitEvent(s2, c->ev_mill[k], 0));   // slot k free again
    int r = light(S, q, off, m, s2);
    if (r) return r;
    HIPCHK(hipEventRecord(c->ev_light[k], s2));
    HIPCHK(hipStreamWaitEvent(s, c->ev_light[k], 0));
    r = heavy(S, q, off, m);
    if (r) return r;
  }
  return CESS_BLS_OK;
}

// Enqueue the verification pipeline for one chunk of n <= cap records.
// sigs/pks/msgs/offs/codes/bitmap/pre are device pointers; gt (optional).
// offs are rebased to msgs; bitmap word 0 covers record 0 of the chunk.
int cess_host::run_chunk(cess_bls_ctx* c, hipStream_t s, uint64_t n, const uint8_t* sigs, const uint8_t* pks,
                         const uint8_t* msgs, const uint64_t* offs, const uint8_t* pre, uint8_t* codes,
                         uint64_t* bitmap, uint8_t* gt) {
  // per-record key buffers (19.6 KB of line coefficients per signature) are
  // allocated on first use: keyed batches never touch them
  for (int k = 0; k < (n > c->qcap ? 2 : 1); k++)
    if (c->slot[k].inf.ensure(c->qcap) | c->slot[k].sig_aff.ensure(c->qcap * CESS_W_G1 * 4) |
        c->slot[k].h_aff.ensure(c->qcap * CESS_W_G1 * 4) | c->slot[k].pk_aff.ensure(c->qcap * CESS_W_G2 * 4) |
        c->slot[k].coeffs.ensure(c->qcap * (uint64_t)CESS_W_COEFFS * 4))
      return CESS_BLS_E_OOM;
  const uint32_t strict = (c->flags & CESS_BLS_F_STRICT_IDENTITY) ? 1u : 0u;
  if (n <= c->small) {
    // small batch: decode + hash one lane per record, then one wave per record
    // runs the Miller loop with the key's lines, the key's subgroup check and
    // the final exponentiation (k_group)
    // (the three light kernels are independent here: the key's code goes to
    // code2 and k_group applies the reference precedence; they run on three
    // streams, so a small batch costs the slowest of them, not their sum)
    StageSlot& S = c->slot[0];
    const uint64_t q = c->qcap;
    const unsigned g = grid_for(n);
    uint8_t* inf = S.inf.as<uint8_t>();
    if (c->code2.ensure(q) | c->inf2.ensure(q)) return CESS_BLS_E_OOM;
    uint8_t *code2 = c->code2.as<uint8_t>(), *inf2 = c->inf2.as<uint8_t>();
    hipStream_t s2 = c->stream2, s3 = c->stream3;
    HIPCHK(hipEventRecord(c->ev_start, s));
    HIPCHK(hipStreamWaitEvent(s2, c->ev_start, 0));
    HIPCHK(hipStreamWaitEvent(s3, c->ev_start, 0));
    LAUNCH(ST_DECODE_SIG, s, k_decode_sig, dim3(g), dim3(kBlock), 0, s, n, sigs, pre, codes, inf,
           S.sig_aff.as<uint32_t>(), q);
    HIPCHK(hipMemsetAsync(code2, 0, n, s2));
    HIPCHK(hipMemsetAsync(inf2, 0, n, s2));
    LAUNCH(ST_DECODE_PK, s2, k_decode_pk, dim3(g), dim3(kBlock), 0, s2, n, pks, pre, code2, inf2,
           S.pk_aff.as<uint32_t>(), q, strict);
    LAUNCH(ST_HASH, s3, k_hash, dim3(g), dim3(kBlock), 0, s3, n, msgs, offs, (const uint8_t*)nullptr,
           S.h_aff.as<uint32_t>(), q);
    HIPCHK(hipEventRecord(c->ev_light[0], s2));
    HIPCHK(hipEventRecord(c->ev_light[1], s3));
    HIPCHK(hipStreamWaitEvent(s, c->ev_light[0], 0));
    HIPCHK(hipStreamWaitEvent(s, c->ev_light[1], 0));
    LAUNCH(ST_GROUP, s, k_group, dim3((unsigned)n), dim3(64), 0, s, n, (const uint8_t*)codes, (const uint8_t*)inf,
           (const uint8_t*)code2, (const uint8_t*)inf2, (const uint32_t*)S.sig_aff.as<uint32_t>(),
           (const uint32_t*)S.h_aff.as<uint32_t>(), (const uint32_t*)S.pk_aff.as<uint32_t>(), q, codes, gt);
    hipLaunchKernelGGL(k_codes_bitmap, dim3(g), dim3(kBlock), 0, s, n, (const uint8_t*)codes, bitmap);
    HIPCHK(hipGetLastError());
    return CESS_BLS_OK;
  }
  auto light = [&](StageSlot& S, uint64_t q, uint64_t off, uint64_t m, hipStream_t t) -> int {
    const unsigned g = grid_for(m);
    uint8_t* inf = S.inf.as<uint8_t>();
    const uint8_t* p = pre ? pre + off : nullptr;
    LAUNCH(ST_DECODE_SIG, t, k_decode_sig, dim3(g), dim3(kBlock), 0, t, m, sigs + 48 * off, p, codes + off, inf,
           S.sig_aff.as<uint32_t>(), q);
    LAUNCH(ST_DECODE_PK, t, k_decode_pk, dim3(g), dim3(kBlock), 0, t, m, pks + 96 * off, p, codes + off, inf,
           S.pk_aff.as<uint32_t>(), q, strict);
    LAUNCH(ST_HASH, t, k_hash, dim3(g), dim3(kBlock), 0, t, m, msgs, offs + off, (const uint8_t*)(codes + off),
           S.h_aff.as<uint32_t>(), q);
    LAUNCH(ST_PREPARE, t, k_prepare, dim3(g), dim3(kBlock), 0, t, m, (const uint32_t*)S.pk_aff.as<uint32_t>(),
           S.coeffs.as<uint4>(), q, codes + off, (const uint8_t*)inf);
    HIPCHK(hipGetLastError());
    return CESS_BLS_OK;
  };
  auto heavy = [&](StageSlot& S, uint64_t q, uint64_t off, uint64_t m) -> int {
    const unsigned g = grid_for(m);
    LAUNCH(ST_MILLER, s, miller_kernel(), miller_grid(m), miller_block(), 0, s, m, (const uint8_t*)(codes + off),
           (const uint8_t*)S.inf.as<uint8_t>(), (const uint32_t*)S.sig_aff.as<uint32_t>(),
           (const uint32_t*)S.h_aff.as<uint32_t>(), (const uint32_t*)c->neg_g2.as<uint32_t>(),
           (const uint4*)S.coeffs.as<uint4>(), c->fval.as<uint4>(), c->fe_slots.as<uint4>(), q,
           (const uint32_t*)nullptr, q, (const uint8_t*)nullptr);
    if (n > c->qcap) HIPCHK(hipEventRecord(c->ev_mill[(off / c->qcap) & 1], s));
    LAUNCH(ST_FINAL, s, final_kernel(), final_grid(m), final_block(), 0, s, m, codes + off, c->fval.as<uint4>(),
           c->fe_slots.as<uint4>(), bitmap + off / 64, gt ? gt + 576 * off : (uint8_t*)nullptr, q);
    HIPCHK(hipGetLastError());
    return CESS_BLS_OK;
  };
  return pipeline(c, s, n, light, heavy);
}

int cess_host::collect_profile(cess_bls_ctx* c, hipStream_t s) {
  if (!(c->flags & CESS_BLS_F_PROFILE)) return CESS_BLS_OK;
  HIPCHK(hipStreamSynchronize(s));
  HIPCHK(hipStreamSynchronize(c->stream2));
  HIPCHK(hipStreamSynchronize(c->stream3));
  for (const ProfRec& p : c->prof) {
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, p.a, p.b));
    c->stage_ms[p.stage] += ms;
    c->stage_launches[p.stage]++;
  }
  c->prof.clear();
  c->evused = 0;
  return CESS_BLS_OK;
}

// Host-buffer batch over fixed-stride inputs (pre: optional host pre-flags).
// msg offsets are absolute into msgs; each chunk is rebased.
int cess_host::verify_host(cess_bls_ctx* c, size_t n, const uint8_t* sigs, const uint8_t* pks, const uint8_t* msgs,
                           const uint64_t* offs, const uint8_t* pre, uint8_t* codes_out, uint64_t* bitmap_out,
                           uint8_t* gt_out) {
  if (n == 0) return CESS_BLS_OK;
  if (!sigs || !pks || !offs || (!msgs && offs[n] != offs[0])) return CESS_BLS_E_INVALID_ARG;
  HIPCHK(hipSetDevice(c->device));
  hipStream_t s = c->stream;
  int r = order_begin(c, s);
  if (r) return r;
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
    r = CESS_BLS_OK;
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
  return order_end(c, s);
}

int cess_host::verify_var_host(cess_bls_ctx* c, size_t n, const uint8_t* sig_data, const uint64_t* sig_offsets,
                               const uint8_t* pk_data, const uint64_t* pk_offsets, const uint8_t* msgs,
                               const uint64_t* msg_offsets, uint8_t* codes_out, uint64_t* bitmap_out) {
  if (!sig_offsets || !pk_offsets || !msg_offsets) return CESS_BLS_E_INVALID_ARG;
  if (n == 0) return CESS_BLS_OK;
  // a null record buffer only with all its records empty
  if ((!sig_data && sig_offsets[n] != sig_offsets[0]) || (!pk_data && pk_offsets[n] != pk_offsets[0]))
    return CESS_BLS_E_INVALID_ARG;
  std::vector<uint8_t> sigs(n * 48, 0), pks(n * 96, 0), pre(n, 0);
  for (size_t i = 0; i < n; i++) {
    if (sig_offsets[i + 1] < sig_offsets[i] || pk_offsets[i + 1] < pk_offsets[i]) return CESS_BLS_E_INVALID_ARG;
    uint64_t sl = sig_offsets[i + 1] - sig_offsets[i], pl = pk_offsets[i + 1] - pk_offsets[i];
    if (sl == 48) memcpy(&sigs[48 * i], sig_data + sig_offsets[i], 48);
    else pre[i] |= PRE_SIG_LEN_BAD;
    if (pl == 96) memcpy(&pks[96 * i], pk_data + pk_offsets[i], 96);
    else pre[i] |= PRE_PK_LEN_BAD;
  }
  return verify_host(c, n, sigs.data(), pks.data(), msgs, msg_offsets, pre.data(), codes_out, bitmap_out, nullptr);
}

// multi-device forms (host_multi.cpp)
int cess_multi_verify(cess_bls_ctx* c, size_t n, const uint8_t* sigs, const uint8_t* pks, const uint8_t* msgs,
                      const uint64_t* offs, uint8_t* codes_out, uint64_t* bitmap_out, bool rlc, const uint8_t* seed32,
                      uint64_t* stats4);
int cess_multi_verify_var(cess_bls_ctx* c, size_t n, const uint8_t* sig_data, const uint64_t* sig_offsets,
                          const uint8_t* pk_data, const uint64_t* pk_offsets, const uint8_t* msgs,
                          const uint64_t* msg_offsets, uint8_t* codes_out, uint64_t* bitmap_out);
int cess_multi_keyed(cess_bls_ctx* c, size_t n, const uint8_t* sigs, const uint32_t* key_idx, const uint8_t* msgs,
                     const uint64_t* offs, uint8_t* codes_out, uint64_t* bitmap_out);
int cess_multi_keys_load(cess_bls_ctx* c, size_t k, const uint8_t* pks, uint8_t* key_codes_out);
int cess_multi_gen(cess_bls_ctx* c, int kind, size_t n, const uint8_t* sks, const uint8_t* msgs, const uint64_t* offs,
                   uint8_t* out);
int cess_multi_gt(cess_bls_ctx* c, size_t n, const uint8_t* sigs, const uint8_t* pks, const uint8_t* msgs,
                  const uint64_t* offs, uint8_t* codes_out, uint8_t* gt_out);

#define ENTRY(c)                          \
  if (!(c)) return CESS_BLS_E_INVALID_ARG; \
  CtxLock lock_(c);                        \
  if (!lock_.ok()) return CESS_BLS_E_BUSY

extern "C" int cess_bls_verify_batch(cess_bls_ctx* c, size_t n, const uint8_t* sigs, const uint8_t* pks,
                                     const uint8_t* msgs, const uint64_t* msg_offsets, uint8_t* codes_out,
                                     uint64_t* bitmap_out) {
  ENTRY(c);
  if (!c->subs.empty())
    return cess_multi_verify(c, n, sigs, pks, msgs, msg_offsets, codes_out, bitmap_out, c->mode == CESS_BLS_MODE_RLC,
                             nullptr, nullptr);
  if (c->mode == CESS_BLS_MODE_RLC)
    return verify_rlc_host(c, n, sigs, pks, msgs, msg_offsets, nullptr, codes_out, bitmap_out, nullptr);
  return verify_host(c, n, sigs, pks, msgs, msg_offsets, nullptr, codes_out, bitmap_out, nullptr);
}

extern "C" int cess_bls_gt_batch(cess_bls_ctx* c, size_t n, const uint8_t* sigs, const uint8_t* pks, const uint8_t* msgs,
                                 const uint64_t* msg_offsets, uint8_t* codes_out, uint8_t* gt_out) {
  ENTRY(c);
  if (!gt_out) return CESS_BLS_E_INVALID_ARG;
  if (!c->subs.empty()) return cess_multi_gt(c, n, sigs, pks, msgs, msg_offsets, codes_out, gt_out);
  return verify_host(c, n, sigs, pks, msgs, msg_offsets, nullptr, codes_out, nullptr, gt_out);
}

extern "C" int cess_bls_verify_batch_var(cess_bls_ctx* c, size_t n, const uint8_t* sig_data, const uint64_t* sig_offsets,
                                         const uint8_t* pk_data, const uint64_t* pk_offsets, const uint8_t* msgs,
                                         const uint64_t* msg_offsets, uint8_t* codes_out, uint64_t* bitmap_out) {
  ENTRY(c);
  if (!c->subs.empty())
    return cess_multi_verify_var(c, n, sig_data, sig_offsets, pk_data, pk_offsets, msgs, msg_offsets, codes_out,
                                 bitmap_out);
  return verify_var_host(c, n, sig_data, sig_offsets, pk_data, pk_offsets, msgs, msg_offsets, codes_out, bitmap_out);
}

extern "C" int cess_bls_verify(cess_bls_ctx* c, const uint8_t* sig, size_t sig_len, const uint8_t* msg, size_t msg_len,
                               const uint8_t* key, size_t key_len, uint8_t* code_out) {
  ENTRY(c);
  if (!code_out || (!sig && sig_len) || (!key && key_len) || (!msg && msg_len)) return CESS_BLS_E_INVALID_ARG;
  cess_bls_ctx* d = c->subs.empty() ? c : c->subs[0];
  uint64_t so[2] = {0, sig_len}, po[2] = {0, key_len}, mo[2] = {0, msg_len};
  static const uint8_t zero = 0;
  return verify_var_host(d, 1, sig ? sig : &zero, so, key ? key : &zero, po, msg ? msg : &zero, mo, code_out, nullptr);
}

extern "C" int cess_bls_enclave_verify_bls(cess_bls_ctx* c, const uint8_t* key, size_t key_len, const uint8_t* msg,
                                           size_t msg_len, const uint8_t* sig, size_t sig_len, int* ok_out) {
  ENTRY(c);
  if (!ok_out || (!sig && sig_len) || (!key && key_len) || (!msg && msg_len)) return CESS_BLS_E_INVALID_ARG;
  *ok_out = 0;
  cess_bls_ctx* d = c->subs.empty() ? c : c->subs[0];
  // record 0 classifies the key alone (paired with the identity signature, a
  // valid encoding), record 1 is the full verification; the key's verdict is
  // taken first, as PublicKey::deserialize(key).unwrap() runs first (:231)
  static const uint8_t zero = 0;
  uint8_t id_sig[48] = {0xc0};
  std::vector<uint8_t> sd(48 + sig_len), kd(2 * key_len + 1), md(msg_len + 1);
  memcpy(sd.data(), id_sig, 48);
  if (sig_len) memcpy(sd.data() + 48, sig, sig_len);
  if (key_len) {
    memcpy(kd.data(), key, key_len);
    memcpy(kd.data() + key_len, key, key_len);
  }
  if (msg_len) memcpy(md.data(), msg, msg_len);
  uint64_t so[3] = {0, 48, 48 + sig_len}, po[3] = {0, key_len, 2 * key_len}, mo[3] = {0, 0, msg_len};
  uint8_t codes[2] = {0xff, 0xff};
  int r = verify_var_host(d, 2, sd.data(), so, key_len ? kd.data() : &zero, po, msg_len ? md.data() : &zero, mo, codes,
                          nullptr);
  if (r) return r;
  if (codes[0] == CODE_PK_LEN || codes[0] == CODE_PK_POINT) return CESS_BLS_E_BAD_KEY;
  if (codes[1] == CODE_SIG_LEN || codes[1] == CODE_SIG_POINT) return CESS_BLS_E_BAD_SIG;
  *ok_out = codes[1] == CODE_OK;
  return CESS_BLS_OK;
}

extern "C" int cess_bls_verify_batch_device(cess_bls_ctx* c, size_t n, const uint8_t* d_sigs, const uint8_t* d_pks,
                                            const uint8_t* d_msgs, const uint64_t* d_offs, uint8_t* d_codes,
                                            uint64_t* d_bitmap, void* stream) {
  ENTRY(c);
  if (!c->subs.empty() || !d_sigs || !d_pks || !d_offs || !d_codes) return CESS_BLS_E_INVALID_ARG;
  HIPCHK(hipSetDevice(c->device));
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  int r = order_begin(c, s);
  if (r) return r;
  for (size_t off = 0; off < n; off += c->cap) {
    uint64_t m = std::min<uint64_t>(c->cap, n - off);
    r = run_chunk(c, s, m, d_sigs + 48 * off, d_pks + 96 * off, d_msgs, d_offs + off, nullptr, d_codes + off,
                  d_bitmap ? d_bitmap + off / 64 : c->bitmap.as<uint64_t>(), nullptr);
    if (r) return r;
    if (c->flags & CESS_BLS_F_PROFILE) {
      r = collect_profile(c, s);
      if (r) return r;
    }
  }
  return order_end(c, s);
}

// distinct-key table ---------------------------------------------------------
// Per-key work of PublicKey::deserialize (src/lib.rs:68-82) and
// G2Prepared::from (:88) done once per distinct key (SURVEY §8(a) A5/A11:
// "cacheable per distinct pk"); the keyed batches then index the table.
int cess_keys_load_one(cess_bls_ctx* c, size_t k, const uint8_t* pks, uint8_t* key_codes_out) {
  if ((k && !pks) || k > 0xffffffffull) return CESS_BLS_E_INVALID_ARG;
  HIPCHK(hipSetDevice(c->device));
  hipStream_t s = c->stream;
  int r = order_begin(c, s);
  if (r) return r;
  c->nkeys = 0;
  if (k == 0) return CESS_BLS_OK;
  r = c->key_in.ensure(k * 96) | c->key_code.ensure(k) | c->key_inf.ensure(k) | c->key_aff.ensure(k * CESS_W_G2 * 4) |
      c->key_coeffs.ensure(k * (uint64_t)CESS_W_COEFFS * 4) | c->key_norm.ensure(k);
  if (r) return CESS_BLS_E_OOM;
  // scratch of k_norm_keys: 68 Fp2 per key, released when the table is built
  DevBuf pre;
  if (pre.ensure(k * 68ull * 24 * 4)) return CESS_BLS_E_OOM;
  HIPCHK(hipMemcpyAsync(c->key_in.p, pks, k * 96, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemsetAsync(c->key_code.p, 0, k, s));
  HIPCHK(hipMemsetAsync(c->key_inf.p, 0, k, s));
  const uint32_t strict = (c->flags & CESS_BLS_F_STRICT_IDENTITY) ? 1u : 0u;
  hipLaunchKernelGGL(k_decode_pk, dim3(grid_for(k)), dim3(kBlock), 0, s, (uint64_t)k, c->key_in.as<uint8_t>(),
                     (const uint8_t*)nullptr, c->key_code.as<uint8_t>(), c->key_inf.as<uint8_t>(),
                     c->key_aff.as<uint32_t>(), (uint64_t)k, strict);
  hipLaunchKernelGGL(k_prepare, dim3(grid_for(k)), dim3(kBlock), 0, s, (uint64_t)k,
                     (const uint32_t*)c->key_aff.as<uint32_t>(), c->key_coeffs.as<uint4>(), (uint64_t)k,
                     c->key_code.as<uint8_t>(), (const uint8_t*)c->key_inf.as<uint8_t>());
  // every signature of a key reuses its lines: normalise them once (the
  // keyed Miller loop then costs 9 Fp2 products per key line instead of 13)
  hipLaunchKernelGGL(k_norm_keys, dim3(grid_for(k)), dim3(kBlock), 0, s, (uint64_t)k, (uint64_t)k, c->key_coeffs.as<uint4>(),
                     pre.as<uint32_t>(), c->key_norm.as<uint8_t>());
  HIPCHK(hipGetLastError());
  if (key_codes_out) HIPCHK(hipMemcpyAsync(key_codes_out, c->key_code.p, k, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  c->nkeys = (uint32_t)k;
  return order_end(c, s);
}

extern "C" int cess_bls_keys_load(cess_bls_ctx* c, size_t k, const uint8_t* pks, uint8_t* key_codes_out) {
  ENTRY(c);
  if (!c->subs.empty()) return cess_multi_keys_load(c, k, pks, key_codes_out);
  return cess_keys_load_one(c, k, pks, key_codes_out);
}

// One chunk of a keyed batch: sig decode, key verdicts from the table, hash,
// Miller loop over the table's coefficient rows, final exponentiation.
static int run_chunk_keyed(cess_bls_ctx* c, hipStream_t s, uint64_t n, const uint8_t* sigs, const uint32_t* idx,
                           const uint8_t* msgs, const uint64_t* offs, uint8_t* codes, uint64_t* bitmap) {
  for (int k = 0; k < (n > c->qcap ? 2 : 1); k++)
    if (c->slot[k].inf.ensure(c->qcap) | c->slot[k].sig_aff.ensure(c->qcap * CESS_W_G1 * 4) |
        c->slot[k].h_aff.ensure(c->qcap * CESS_W_G1 * 4))
      return CESS_BLS_E_OOM;
  auto light = [&](StageSlot& S, uint64_t q, uint64_t off, uint64_t m, hipStream_t t) -> int {
    const unsigned g = grid_for(m);
    uint8_t* inf = S.inf.as<uint8_t>();
    LAUNCH(ST_DECODE_SIG, t, k_decode_sig, dim3(g), dim3(kBlock), 0, t, m, sigs + 48 * off, (const uint8_t*)nullptr,
           codes + off, inf, S.sig_aff.as<uint32_t>(), q);
    LAUNCH(ST_DECODE_PK, t, k_merge_pk, dim3(g), dim3(kBlock), 0, t, m, idx + off, c->nkeys,
           (const uint8_t*)c->key_code.as<uint8_t>(), (const uint8_t*)c->key_inf.as<uint8_t>(), codes + off, inf);
    LAUNCH(ST_HASH, t, k_hash, dim3(g), dim3(kBlock), 0, t, m, msgs, offs + off, (const uint8_t*)(codes + off),
           S.h_aff.as<uint32_t>(), q);
    HIPCHK(hipGetLastError());
    return CESS_BLS_OK;
  };
  auto heavy = [&](StageSlot& S, uint64_t q, uint64_t off, uint64_t m) -> int {
    const unsigned g = grid_for(m);
    LAUNCH(ST_MILLER, s, miller_kernel(), miller_grid(m), miller_block(), 0, s, m, (const uint8_t*)(codes + off),
           (const uint8_t*)S.inf.as<uint8_t>(), (const uint32_t*)S.sig_aff.as<uint32_t>(),
           (const uint32_t*)S.h_aff.as<uint32_t>(), (const uint32_t*)c->neg_g2.as<uint32_t>(),
           (const uint4*)c->key_coeffs.as<uint4>(), c->fval.as<uint4>(), c->fe_slots.as<uint4>(), q, idx + off,
           (uint64_t)c->nkeys, (const uint8_t*)c->key_norm.as<uint8_t>());
    if (n > c->qcap) HIPCHK(hipEventRecord(c->ev_mill[(off / c->qcap) & 1], s));
    LAUNCH(ST_FINAL, s, final_kernel(), final_grid(m), final_block(), 0, s, m, codes + off, c->fval.as<uint4>(),
           c->fe_slots.as<uint4>(), bitmap + off / 64, (uint8_t*)nullptr, q);
    HIPCHK(hipGetLastError());
    return CESS_BLS_OK;
  };
  return pipeline(c, s, n, light, heavy);
}

extern "C" int cess_bls_verify_batch_keyed_device(cess_bls_ctx* c, size_t n, const uint8_t* d_sigs,
                                                  const uint32_t* d_key_idx, const uint8_t* d_msgs,
                                                  const uint64_t* d_offs, uint8_t* d_codes, uint64_t* d_bitmap,
                                                  void* stream) {
  ENTRY(c);
  if (!c->subs.empty() || !d_sigs || !d_key_idx || !d_offs || !d_codes) return CESS_BLS_E_INVALID_ARG;
  if (n == 0) return CESS_BLS_OK;
  if (c->nkeys == 0) return CESS_BLS_E_INVALID_ARG;
  HIPCHK(hipSetDevice(c->device));
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  int r = order_begin(c, s);
  if (r) return r;
  for (size_t off = 0; off < n; off += c->cap) {
    uint64_t m = std::min<uint64_t>(c->cap, n - off);
    r = run_chunk_keyed(c, s, m, d_sigs + 48 * off, d_key_idx + off, d_msgs, d_offs + off, d_codes + off,
                        d_bitmap ? d_bitmap + off / 64 : c->bitmap.as<uint64_t>());
    if (r) return r;
    r = collect_profile(c, s);
    if (r) return r;
  }
  return order_end(c, s);
}

int cess_keyed_one(cess_bls_ctx* c, size_t n, const uint8_t* sigs, const uint32_t* key_idx, const uint8_t* msgs,
                   const uint64_t* offs, uint8_t* codes_out, uint64_t* bitmap_out) {
  if (n == 0) return CESS_BLS_OK;
  if (!sigs || !key_idx || !offs || (!msgs && offs[n] != offs[0])) return CESS_BLS_E_INVALID_ARG;
  if (c->nkeys == 0) return CESS_BLS_E_INVALID_ARG;
  // an out-of-range key index is a caller error on the host-buffer API
  for (size_t i = 0; i < n; i++)
    if (key_idx[i] >= c->nkeys) return CESS_BLS_E_INVALID_ARG;
  HIPCHK(hipSetDevice(c->device));
  hipStream_t s = c->stream;
  int r = order_begin(c, s);
  if (r) return r;
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
    r = c->in_sigs.ensure(m * 48) | c->in_idx.ensure(m * 4) | c->in_msgs.ensure(std::max<uint64_t>(mb1 - mb0, 1)) |
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
  return order_end(c, s);
}

extern "C" int cess_bls_verify_batch_keyed(cess_bls_ctx* c, size_t n, const uint8_t* sigs, const uint32_t* key_idx,
                                           const uint8_t* msgs, const uint64_t* offs, uint8_t* codes_out,
                                           uint64_t* bitmap_out) {
  ENTRY(c);
  if (!c->subs.empty()) return cess_multi_keyed(c, n, sigs, key_idx, msgs, offs, codes_out, bitmap_out);
  return cess_keyed_one(c, n, sigs, key_idx, msgs, offs, codes_out, bitmap_out);
}

// generator-side batches -----------------------------------------------------
int cess_gen_one(cess_bls_ctx* c, int kind, size_t n, const uint8_t* sks, const uint8_t* msgs, const uint64_t* offs,
                 uint8_t* out) {
  if (!out) return CESS_BLS_E_INVALID_ARG;
  if (n == 0) return CESS_BLS_OK;
  HIPCHK(hipSetDevice(c->device));
  hipStream_t s = c->stream;
  int r = order_begin(c, s);
  if (r) return r;
  const size_t ob = kind == 0 ? 96 : 48;
  std::vector<uint64_t> rebased;
  for (size_t off = 0; off < n; off += c->cap) {
    uint64_t m = std::min<uint64_t>(c->cap, n - off);
    r = c->out_bytes.ensure(m * ob);
    if (kind != 2) r |= c->in_sks.ensure(m * 32);
    if (r) return CESS_BLS_E_OOM;
    if (kind != 2) HIPCHK(hipMemcpyAsync(c->in_sks.p, sks + 32 * off, m * 32, hipMemcpyHostToDevice, s));
    if (kind != 0) {
      uint64_t mb0 = offs[off], mb1 = offs[off + m];
      if (mb1 < mb0) return CESS_BLS_E_INVALID_ARG;
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
  return order_end(c, s);
}

static int gen_batch(cess_bls_ctx* c, int kind, size_t n, const uint8_t* sks, const uint8_t* msgs, const uint64_t* offs,
                     uint8_t* out) {
  if (!c->subs.empty()) return cess_multi_gen(c, kind, n, sks, msgs, offs, out);
  return cess_gen_one(c, kind, n, sks, msgs, offs, out);
}

extern "C" int cess_bls_public_key_batch(cess_bls_ctx* c, size_t n, const uint8_t* sks, uint8_t* pks_out) {
  ENTRY(c);
  if (!sks && n) return CESS_BLS_E_INVALID_ARG;
  return gen_batch(c, 0, n, sks, nullptr, nullptr, pks_out);
}
extern "C" int cess_bls_sign_batch(cess_bls_ctx* c, size_t n, const uint8_t* sks, const uint8_t* msgs,
                                   const uint64_t* offs, uint8_t* sigs_out) {
  ENTRY(c);
  if ((!sks || !offs) && n) return CESS_BLS_E_INVALID_ARG;
  return gen_batch(c, 1, n, sks, msgs, offs, sigs_out);
}
// PrivateKey::sign over device-resident records (the TEE-side batch signer,
// SURVEY §8(f) rank 3): one k_sign launch, enqueued on `stream`.
extern "C" int cess_bls_sign_batch_device(cess_bls_ctx* c, size_t n, const uint8_t* d_sks, const uint8_t* d_msgs,
                                          const uint64_t* d_offs, uint8_t* d_sigs_out, void* stream) {
  ENTRY(c);
  if (!c->subs.empty() || (n && (!d_sks || !d_offs || !d_sigs_out))) return CESS_BLS_E_INVALID_ARG;
  if (n == 0) return CESS_BLS_OK;
  if (n >= (1ull << 40)) return CESS_BLS_E_INVALID_ARG;
  HIPCHK(hipSetDevice(c->device));
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  int r = order_begin(c, s);
  if (r) return r;
  LAUNCH(ST_SIGN, s, k_sign, dim3(grid_for(n)), dim3(kBlock), 0, s, (uint64_t)n, d_sks, d_msgs, d_offs, d_sigs_out);
  HIPCHK(hipGetLastError());
  if (c->flags & CESS_BLS_F_PROFILE) {
    r = collect_profile(c, s);
    if (r) return r;
  }
  return order_end(c, s);
}

extern "C" int cess_bls_hash_to_g1_batch(cess_bls_ctx* c, size_t n, const uint8_t* msgs, const uint64_t* offs,
                                         uint8_t* out48) {
  ENTRY(c);
  if (!offs && n) return CESS_BLS_E_INVALID_ARG;
  return gen_batch(c, 2, n, nullptr, msgs, offs, out48);
}

extern "C" int cess_bls_stage_stats(cess_bls_ctx* c, const char** names, double* ms, uint64_t* launches, int max,
                                    int reset) {
  ENTRY(c);
  int k = std::min(max, (int)ST_N);
  for (int i = 0; i < k; i++) {
    double v = c->stage_ms[i];
    uint64_t l = c->stage_launches[i];
    for (cess_bls_ctx* s : c->subs) v += s->stage_ms[i], l += s->stage_launches[i];
    if (names) names[i] = kStageNames[i];
    if (ms) ms[i] = v;
    if (launches) launches[i] = l;
  }
  if (reset) {
    for (int i = 0; i < ST_N; i++) c->stage_ms[i] = 0, c->stage_launches[i] = 0;
    for (cess_bls_ctx* s : c->subs)
      for (int i = 0; i < ST_N; i++) s->stage_ms[i] = 0, s->stage_launches[i] = 0;
  }
  return ST_N;
}

extern "C" int cess_bls_stage_times(cess_bls_ctx* c, const char** names, double* ms, int max, int reset) {
  return cess_bls_stage_stats(c, names, ms, nullptr, max, reset);
}

extern "C" uint64_t cess_bls_launch_records(cess_bls_ctx* c) { return c ? c->qcap : 0; }

// device memory helpers -------------------------------------------------------
extern "C" int cess_bls_device_alloc(cess_bls_ctx* c, size_t bytes, void** d_out) {
  if (!c || !d_out || !c->subs.empty()) return CESS_BLS_E_INVALID_ARG;
  *d_out = nullptr;
  HIPCHK(hipSetDevice(c->device));
  if (hipMalloc(d_out, std::max<size_t>(bytes, 1)) != hipSuccess) return CESS_BLS_E_OOM;
  return CESS_BLS_OK;
}
extern "C" int cess_bls_device_free(cess_bls_ctx* c, void* d) {
  if (!c || !c->subs.empty()) return CESS_BLS_E_INVALID_ARG;
  if (!d) return CESS_BLS_OK;
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipStreamSynchronize(c->stream));
  HIPCHK(hipFree(d));
  return CESS_BLS_OK;
}
extern "C" int cess_bls_copy_to_device(cess_bls_ctx* c, void* d_dst, const void* src, size_t bytes) {
  ENTRY(c);
  if (!c->subs.empty() || (bytes && (!d_dst || !src))) return CESS_BLS_E_INVALID_ARG;
  HIPCHK(hipSetDevice(c->device));
  int r = order_begin(c, c->stream);
  if (r) return r;
  if (bytes) HIPCHK(hipMemcpyAsync(d_dst, src, bytes, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return order_end(c, c->stream);
}
extern "C" int cess_bls_copy_from_device(cess_bls_ctx* c, void* dst, const void* d_src, size_t bytes) {
  ENTRY(c);
  if (!c->subs.empty() || (bytes && (!dst || !d_src))) return CESS_BLS_E_INVALID_ARG;
  HIPCHK(hipSetDevice(c->device));
  int r = order_begin(c, c->stream);
  if (r) return r;
  if (bytes) HIPCHK(hipMemcpyAsync(dst, d_src, bytes, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return order_end(c, c->stream);
}
extern "C" int cess_bls_synchronize(cess_bls_ctx* c) {
  ENTRY(c);
  for (cess_bls_ctx* s : c->subs) {
    HIPCHK(hipSetDevice(s->device));
    HIPCHK(hipDeviceSynchronize());
  }
  if (c->subs.empty()) {
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipDeviceSynchronize());
  }
  return CESS_BLS_OK;
}
