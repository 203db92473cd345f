// RLC batch mode (north_star "optional random-linear-combination batch mode";
// SURVEY §8(d) C4, §8(e)).  One random linear combination per (sub)batch; on
// failure the batch is bisected down to leaves of kRlcLeaf records, which are
// verified per signature, so the final codes are those of
// cess_bls_verify_batch (up to the 2^-127 soundness error per check).
#include <string.h>
#include <sys/random.h>

#include <thread>

#include "host.hpp"

using namespace cess_host;

namespace {
constexpr uint64_t kRlcLeaf = 2048;

// per-kernel HIP-event records of the RLC path's chunk kernels (with
// CESS_BLS_F_PROFILE; host.cpp LAUNCH): bench.py's RLC lines take their
// roofline from these (the Miller stage is k_miller_rr in the distinct-key mode)
#define RLAUNCH(stage, strm, ...)                        \
  do {                                                   \
    hipEvent_t pa_;                                      \
    int pr_ = prof_begin(c, strm, stage, &pa_);          \
    if (pr_) return pr_;                                 \
    hipLaunchKernelGGL(__VA_ARGS__);                     \
    pr_ = prof_end(c, strm, stage, pa_);                 \
    if (pr_) return pr_;                                 \
  } while (0)   // records verified per signature
constexpr uint64_t kRlcFan = 16;      // bisection fan-out per level
// distinct-key mode: a level re-multiplies stored Miller values and costs one
// single-wave Miller loop and final exponentiation of latency whatever its
// range count, so fewer, wider levels
constexpr uint64_t kRlcdFan = 64;
constexpr uint64_t kProdLanes = 64;   // lanes per range in the Fp12 segment product

// one (range, key group) term of a batched check: perm positions [lo, hi)
struct Term {
  uint32_t range, group;
  uint64_t lo, hi;
};
}  // namespace

int cess_host::os_random(uint8_t* out, size_t n) {
  size_t got = 0;
  while (got < n) {
    ssize_t r = getrandom(out + got, n - got, 0);
    if (r <= 0) return CESS_BLS_E_INVALID_ARG;
    got += (size_t)r;
  }
  return CESS_BLS_OK;
}

// Segmented sums: out[s] (stride out_stride) = sum of in[perm[off_s + j]], j < cnt_s.
// Two passes of k_g1_sum_segs (B partial sums per segment, then one).
static int rlc_sums(RlcState& R, hipStream_t s, const std::vector<uint64_t>& off, const std::vector<uint64_t>& cnt,
                    const uint32_t* in, uint64_t in_stride, uint32_t* out, uint64_t out_stride) {
  const uint64_t ns = off.size();
  if (ns == 0) return CESS_BLS_OK;
  uint64_t mx = 1;
  for (uint64_t v : cnt) mx = std::max(mx, v);
  const uint64_t B = std::max<uint64_t>(1, std::min<uint64_t>(std::max<uint64_t>(1, 1024 / ns), (mx + 255) / 256));
  std::vector<uint64_t> h(4 * ns);
  for (uint64_t q = 0; q < ns; q++) h[q] = off[q], h[ns + q] = cnt[q], h[2 * ns + q] = q * B, h[3 * ns + q] = B;
  if (B * ns >= (1ull << 31)) return CESS_BLS_E_INVALID_ARG;
  if (R.seg.ensure(h.size() * 8) || R.part.ensure(ns * B * 36 * 4)) return CESS_BLS_E_OOM;
  HIPCHK(hipMemcpyAsync(R.seg.p, h.data(), h.size() * 8, hipMemcpyHostToDevice, s));
  const uint64_t* d = R.seg.as<uint64_t>();
  hipLaunchKernelGGL(k_g1_sum_segs, dim3((unsigned)(B * ns)), dim3(256), 0, s, (uint32_t)B, d, d + ns,
                     (const uint32_t*)R.d_perm.as<uint32_t>(), in, in_stride, R.part.as<uint32_t>(), ns * B);
  hipLaunchKernelGGL(k_g1_sum_segs, dim3((unsigned)ns), dim3(256), 0, s, 1u, d + 2 * ns, d + 3 * ns,
                     (const uint32_t*)nullptr, (const uint32_t*)R.part.as<uint32_t>(), ns * B, out, out_stride);
  HIPCHK(hipGetLastError());
  // the host vector h must outlive the async copy
  HIPCHK(hipStreamSynchronize(s));
  return CESS_BLS_OK;
}

// Open-addressing table of distinct 96-byte keys (ids in insertion order).
struct KeyTable {
  const uint8_t* pks;
  std::vector<uint64_t> first;       // record index of each id's first occurrence
  std::vector<uint32_t> slot = std::vector<uint32_t>(64, 0);   // id + 1; 0 = empty
  uint64_t mask = 63;
  static uint64_t khash(const uint8_t* k) {
    uint64_t h = 0x9E3779B97F4A7C15ull;
    for (int q = 0; q < 96; q += 8) {
      uint64_t w;
      memcpy(&w, k + q, 8);
      h = (h ^ w) * 0xff51afd7ed558ccdull;
      h ^= h >> 29;
    }
    return h;
  }
  // id of record i's key, inserting it (first occurrence i) if new
  uint32_t id(uint64_t i) {
    const uint8_t* k = pks + 96 * i;
    uint64_t h = khash(k) & mask;
    while (slot[h] && memcmp(pks + 96 * first[slot[h] - 1], k, 96) != 0) h = (h + 1) & mask;
    if (slot[h]) return slot[h] - 1;
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
    return (uint32_t)first.size() - 1;
  }
};

// grp[i] = group of record i's key, groups numbered by first occurrence;
// first[g] = that record.  Up to 16 host threads over contiguous slices.
static void group_keys(const uint8_t* pks, uint64_t n, std::vector<uint32_t>& grp, std::vector<uint64_t>& first) {
  const uint64_t T = std::max<uint64_t>(1, std::min<uint64_t>(16, n / 65536));
  std::vector<KeyTable> loc(T, KeyTable{pks});
  std::vector<std::thread> th;
  auto run = [&](uint64_t t) {
    for (uint64_t i = n * t / T; i < n * (t + 1) / T; i++) grp[i] = loc[t].id(i);
  };
  for (uint64_t t = 1; t < T; t++) th.emplace_back(run, t);
  run(0);
  for (auto& x : th) x.join();
  KeyTable glob{pks};
  std::vector<std::vector<uint32_t>> remap(T);
  for (uint64_t t = 0; t < T; t++)
    for (uint64_t f : loc[t].first) remap[t].push_back(glob.id(f));
  first.swap(glob.first);
  if (T == 1) return;   // one slice: its ids are the global ids already
  th.clear();
  auto rm = [&](uint64_t t) {
    for (uint64_t i = n * t / T; i < n * (t + 1) / T; i++) grp[i] = remap[t][grp[i]];
  };
  for (uint64_t t = 1; t < T; t++) th.emplace_back(rm, t);
  rm(0);
  for (auto& x : th) x.join();
}

// Bucket sums (k_rlc.hip, k_msm_*).  env CESS_BLS_RLC_MSM = 0: never (each
// record's multiples P_i, Q_i as before), 1: for every check whose segment
// count fits the tables; default: also at least 64 covered records per
// segment (a segment costs ~4,096 bucket combinations, a record ~32 additions
// against one 128-bit multiple per point).
static int msm_env() {
  const char* e = getenv("CESS_BLS_RLC_MSM");
  return e && e[0] == '0' ? 0 : e && e[0] == '1' ? 1 : 2;
}
static bool msm_ok(uint64_t covered, uint64_t segs) {
  const int e = msm_env();
  if (e == 0 || segs == 0 || segs > CESS_MSM_MAX_SEGS || 32 * covered >= (1ull << 32)) return false;
  return e == 1 || covered >= 64 * segs;
}

// Final exponentiation + identity test of a check's NR products (R.acc,
// stride NR) into R.fin_code (and R.gt when gt): one WAVE per product
// (k_group_fe, the lane-group program: a check's latency is one value's final
// exponentiation, ~10 ms for one lane of k_final), or env CESS_BLS_RLC_FE=lane
// one lane per product (k_final; tests compare the two).
static bool rlc_fe_lane() {
  const char* e = getenv("CESS_BLS_RLC_FE");
  return e && strcmp(e, "lane") == 0;
}
static int rlc_final_exp(cess_bls_ctx* c, RlcState& R, uint64_t NR, hipStream_t s, bool gt) {
  if (rlc_fe_lane()) {
    HIPCHK(hipMemsetAsync(R.fin_code.p, 0, NR, s));
    hipLaunchKernelGGL(k_final, dim3(grid_for(NR)), dim3(kBlock), 0, s, NR, R.fin_code.as<uint8_t>(), R.acc.as<uint4>(),
                       R.slots.as<uint4>(), R.tmp.as<uint64_t>(), gt ? R.gt.as<uint8_t>() : (uint8_t*)nullptr, NR);
  } else {
    hipLaunchKernelGGL(k_group_fe, dim3((unsigned)NR), dim3(64), 0, s, (uint32_t)NR, (const uint4*)R.acc.as<uint4>(),
                       R.fin_code.as<uint8_t>(), gt ? R.gt.as<uint8_t>() : (uint8_t*)nullptr);
  }
  HIPCHK(hipGetLastError());
  return CESS_BLS_OK;
}

// Sums of one check from the batch's points: S[q] = sum_{i in part q} r_i sig_i
// (stride NR), Qs[t] = sum_{i in term t} r_i H_i (stride M), over the records
// with code 0 (identity terms excluded).  Count entries per bucket, lay the
// buckets out (host prefix sums over the counts), scatter the record ids, sum
// each bucket in chunks and the chunks per bucket, then the window running
// sums and the 2^(8w) weights.
static int msm_sums(cess_bls_ctx* c, RlcState& R, const std::vector<std::pair<uint64_t, uint64_t>>& parts,
                    const std::vector<Term>& terms, uint32_t* S, uint32_t* Qs) {
  hipStream_t s = c->stream;
  const uint64_t n = R.n, NR = parts.size(), M = terms.size(), nseg = NR + M, nb = nseg * CESS_MSM_SEG_BUCKETS;
  const uint32_t* seed = R.d_seed.as<uint32_t>();
  // the batch's first check: one part = the batch, term g = group g
  bool first = NR == 1 && parts[0].first == 0 && parts[0].second == n && M == R.K;
  for (uint64_t t = 0; first && t < M; t++) first = terms[t].group == t;
  MsmSegs sg{R.d_grp.as<uint32_t>(), nullptr, nullptr, nullptr, nullptr, nullptr, (uint32_t)NR, (uint32_t)M};
  int r = R.m_cnt.ensure(nb * 4) | R.m_start.ensure(nb * 4) | R.m_cur.ensure(nb * 4) | R.m_items.ensure((nb + 1) * 4);
  r |= R.m_bsum.ensure(nb * 36 * 4) | R.m_T.ensure(nseg * 256 * 36 * 4) | R.m_U.ensure(nseg * 16 * 36 * 4);
  r |= R.m_bounds.ensure(2 * nseg * 4);
  if (!first) r |= R.d_pos.ensure(n * 4);
  if (r) return CESS_BLS_E_OOM;
  std::vector<uint32_t> bounds(2 * nseg);
  if (!first) {
    if (!R.have_pos) {
      hipLaunchKernelGGL(k_inv_perm, dim3(grid_for(n)), dim3(kBlock), 0, s, n, (const uint32_t*)R.d_perm.as<uint32_t>(),
                         R.d_pos.as<uint32_t>());
      R.have_pos = true;
    }
    for (uint64_t q = 0; q < NR; q++) bounds[q] = (uint32_t)parts[q].first, bounds[NR + q] = (uint32_t)parts[q].second;
    for (uint64_t t = 0; t < M; t++)
      bounds[2 * NR + t] = (uint32_t)terms[t].lo, bounds[2 * NR + M + t] = (uint32_t)terms[t].hi;
    HIPCHK(hipMemcpyAsync(R.m_bounds.p, bounds.data(), bounds.size() * 4, hipMemcpyHostToDevice, s));
    const uint32_t* d = R.m_bounds.as<uint32_t>();
    sg = {nullptr, R.d_pos.as<uint32_t>(), d, d + NR, d + 2 * NR, d + 2 * NR + M, (uint32_t)NR, (uint32_t)M};
  }
  HIPCHK(hipMemsetAsync(R.m_cnt.p, 0, nb * 4, s));
  hipLaunchKernelGGL(k_msm_count, dim3(grid_for(n)), dim3(kBlock), 0, s, n, (const uint8_t*)R.d_code.as<uint8_t>(),
                     (const uint8_t*)R.d_inf.as<uint8_t>(), sg, seed, R.index_hi, R.m_cnt.as<uint32_t>());
  HIPCHK(hipGetLastError());
  std::vector<uint32_t> cnt(nb), start(nb), items(nb + 1);
  HIPCHK(hipMemcpyAsync(cnt.data(), R.m_cnt.p, nb * 4, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  uint64_t e = 0, it = 0;
  for (uint64_t b = 0; b < nb; b++) {
    start[b] = (uint32_t)e;
    items[b] = (uint32_t)it;
    e += cnt[b];
    if (cnt[b]) it += (cnt[b] + msm_chunk(cnt[b]) - 1) / msm_chunk(cnt[b]);
  }
  items[nb] = (uint32_t)it;
  if (e >= (1ull << 32) || it >= (1ull << 31)) return CESS_BLS_E_INVALID_ARG;
  if (R.m_idx.ensure(std::max<uint64_t>(e, 1) * 4) || R.m_part.ensure(std::max<uint64_t>(it, 1) * 36 * 4))
    return CESS_BLS_E_OOM;
  HIPCHK(hipMemcpyAsync(R.m_start.p, start.data(), nb * 4, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(R.m_cur.p, start.data(), nb * 4, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(R.m_items.p, items.data(), (nb + 1) * 4, hipMemcpyHostToDevice, s));
  if (e) {
    if (!R.aos) {   // the points record-major, once per batch
      if (R.Xsa.ensure(n * 96) || R.Xha.ensure(n * 96)) return CESS_BLS_E_OOM;
      hipLaunchKernelGGL(k_msm_aos, dim3(grid_for(n)), dim3(kBlock), 0, s, n, (const uint32_t*)R.Xs.as<uint32_t>(),
                         R.Xsa.as<uint4>());
      hipLaunchKernelGGL(k_msm_aos, dim3(grid_for(n)), dim3(kBlock), 0, s, n, (const uint32_t*)R.Xh.as<uint32_t>(),
                         R.Xha.as<uint4>());
      R.aos = true;
    }
    hipLaunchKernelGGL(k_msm_scatter, dim3(grid_for(n)), dim3(kBlock), 0, s, n, (const uint8_t*)R.d_code.as<uint8_t>(),
                       (const uint8_t*)R.d_inf.as<uint8_t>(), sg, seed, R.index_hi, R.m_cur.as<uint32_t>(),
                       R.m_idx.as<uint32_t>());
    hipLaunchKernelGGL(k_msm_items, dim3(grid_for(it)), dim3(kBlock), 0, s, (uint32_t)it, (uint32_t)nb, (uint32_t)NR,
                       (const uint32_t*)R.m_items.as<uint32_t>(), (const uint32_t*)R.m_start.as<uint32_t>(),
                       (const uint32_t*)R.m_cnt.as<uint32_t>(), (const uint32_t*)R.m_idx.as<uint32_t>(),
                       (const uint4*)R.Xsa.as<uint4>(), (const uint4*)R.Xha.as<uint4>(), R.m_part.as<uint32_t>(), it);
  }
  hipLaunchKernelGGL(k_msm_bucket_sum, dim3(grid_for(nb)), dim3(kBlock), 0, s, (uint32_t)nb,
                     (const uint32_t*)R.m_items.as<uint32_t>(), (const uint32_t*)R.m_part.as<uint32_t>(),
                     std::max<uint64_t>(it, 1), R.m_bsum.as<uint32_t>());
  hipLaunchKernelGGL(k_msm_window, dim3(grid_for(nseg * 256)), dim3(kBlock), 0, s, (uint32_t)nseg,
                     (const uint32_t*)R.m_bsum.as<uint32_t>(), nb, R.m_T.as<uint32_t>());
  hipLaunchKernelGGL(k_msm_wsum, dim3(grid_for(nseg * 16)), dim3(kBlock), 0, s, (uint32_t)nseg,
                     (const uint32_t*)R.m_T.as<uint32_t>(), R.m_U.as<uint32_t>());
  hipLaunchKernelGGL(k_msm_finish, dim3(grid_for(nseg)), dim3(kBlock), 0, s, (uint32_t)nseg, (uint32_t)NR,
                     (const uint32_t*)R.m_U.as<uint32_t>(), S, Qs);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(s));   // bounds / start / items are host vectors
  return CESS_BLS_OK;
}

// the per-record multiples P_i = r_i sig_i, Q_i = r_i H_i (a check with too
// many segments for the buckets sums them over its ranges), once per batch
static int rlc_scale_all(cess_bls_ctx* c, RlcState& R) {
  if (R.pq) return CESS_BLS_OK;
  hipStream_t s = c->stream;
  if (R.P.ensure(R.n * 36 * 4) | R.Q.ensure(R.n * 36 * 4)) return CESS_BLS_E_OOM;
  hipLaunchKernelGGL(k_rlc_scale, dim3(grid_for(R.n)), dim3(kBlock), 0, s, R.n, (const uint8_t*)R.d_code.as<uint8_t>(),
                     (const uint8_t*)R.d_inf.as<uint8_t>(), (const uint32_t*)R.Xs.as<uint32_t>(),
                     (const uint32_t*)R.Xh.as<uint32_t>(), (const uint32_t*)R.d_seed.as<uint32_t>(), R.index_hi,
                     R.P.as<uint32_t>(), R.Q.as<uint32_t>(), R.n, R.n, 4u);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(s));
  R.pq = true;
  return CESS_BLS_OK;
}

// RLC checks of NR perm-position ranges in one batch: ok[r] = the product of
// range r's pairings is 1.  Only the (range, key group) terms that intersect
// are formed (perm is sorted by group, so a range meets a contiguous run of
// groups): at most NR + K + NR terms per batch, never NR * K.  gt_out
// (optional, NR == 1): the Gt value of the check.  The sums come from the
// buckets (msm_sums) when the batch's points are on the device and msm_ok,
// else from the per-record multiples.
static int rlc_check_multi(cess_bls_ctx* c, RlcState& R, const std::vector<std::pair<uint64_t, uint64_t>>& rg,
                           std::vector<uint8_t>& ok, uint8_t* gt_out) {
  hipStream_t s = c->stream;
  const uint64_t NR = rg.size();
  R.checks += NR;
  std::vector<Term> terms;
  std::vector<uint64_t> so(NR), sc(NR), tbeg(NR + 1, 0);
  for (uint64_t r = 0; r < NR; r++) {
    const uint64_t a = rg[r].first, b = rg[r].second;
    so[r] = a, sc[r] = b - a;
    tbeg[r] = terms.size();
    if (b > a) {
      // first group with gbeg[g + 1] > a
      uint64_t g = std::upper_bound(R.gbeg.begin(), R.gbeg.end(), a) - R.gbeg.begin() - 1;
      for (; g < R.K && R.gbeg[g] < b; g++) {
        const uint64_t lo = std::max(a, R.gbeg[g]), hi = std::min(b, R.gbeg[g + 1]);
        if (hi > lo) terms.push_back({(uint32_t)r, (uint32_t)g, lo, hi});
      }
    }
  }
  tbeg[NR] = terms.size();
  const uint64_t M = terms.size();
  ok.assign(NR, 1);
  if (M == 0) {
    if (gt_out) {
      memset(gt_out, 0, 576);
      gt_out[47] = 1;
    }
    return CESS_BLS_OK;
  }
  if (M >= (1ull << 31)) return CESS_BLS_E_INVALID_ARG;
  int r = 0;
  r |= R.S.ensure(NR * 36 * 4) | R.Qs.ensure(M * 36 * 4);
  r |= R.rec_code.ensure(M) | R.rec_inf.ensure(M) | R.rec_sig.ensure(M * CESS_W_G1 * 4);
  r |= R.rec_h.ensure(M * CESS_W_G1 * 4) | R.rec_f.ensure(M * CESS_W_FP12 * 4) | R.rec_f2.ensure(M * CESS_W_FP12 * 4);
  r |= R.acc.ensure(NR * CESS_W_FP12 * 4) | R.slots.ensure(NR * CESS_W_FP12 * 4 * CESS_FE_SLOTS);
  r |= R.part2.ensure(NR * kProdLanes * CESS_W_FP12 * 4);
  r |= R.fin_code.ensure(NR) | R.fin_bm.ensure(((NR + 63) / 64) * 8) | R.gt.ensure(NR * 576);
  r |= R.lists.ensure((2 * M + NR + 1) * 4);
  if (r) return CESS_BLS_E_OOM;
  std::vector<uint64_t> qo(M), qc(M);
  std::vector<uint32_t> lists(2 * M + NR + 1);
  for (uint64_t j = 0; j < M; j++) {
    qo[j] = terms[j].lo, qc[j] = terms[j].hi - terms[j].lo;
    lists[j] = terms[j].range;
    lists[M + j] = terms[j].group;
  }
  for (uint64_t q = 0; q <= NR; q++) lists[2 * M + q] = (uint32_t)tbeg[q];
  HIPCHK(hipMemcpyAsync(R.lists.p, lists.data(), lists.size() * 4, hipMemcpyHostToDevice, s));
  const uint32_t* d_range = R.lists.as<uint32_t>();
  const uint32_t* d_group = d_range + M;
  const uint32_t* d_tbeg = d_range + 2 * M;
  uint64_t covered = 0;
  for (uint64_t q = 0; q < NR; q++) covered += sc[q];
  if (R.pts && msm_ok(covered, NR + M)) {
    r = msm_sums(c, R, rg, terms, R.S.as<uint32_t>(), R.Qs.as<uint32_t>());
    if (r) return r;
  } else {
    r = rlc_scale_all(c, R);
    if (r) return r;
    r = rlc_sums(R, s, so, sc, R.P.as<uint32_t>(), R.n, R.S.as<uint32_t>(), NR);
    if (r) return r;
    r = rlc_sums(R, s, qo, qc, R.Q.as<uint32_t>(), R.n, R.Qs.as<uint32_t>(), M);
    if (r) return r;
  }
  hipLaunchKernelGGL(k_rlc_pairs_list, dim3((unsigned)((M + 63) / 64)), dim3(64), 0, s, (uint32_t)M, (uint32_t)NR, d_range, d_group,
                     (const uint32_t*)R.S.as<uint32_t>(), (const uint8_t*)R.pk_usable.as<uint8_t>(),
                     R.rec_code.as<uint8_t>(), R.rec_inf.as<uint8_t>(), R.rec_sig.as<uint32_t>(),
                     R.rec_h.as<uint32_t>(), R.Qs.as<uint32_t>());
  // the Miller loop reads each term's key rows straight from the distinct-key
  // table (cidx = group, table stride K): nothing is replicated
  hipLaunchKernelGGL(k_miller, dim3((unsigned)((M + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, M,
                     (const uint8_t*)R.rec_code.as<uint8_t>(), (const uint8_t*)R.rec_inf.as<uint8_t>(),
                     (const uint32_t*)R.rec_sig.as<uint32_t>(), (const uint32_t*)R.rec_h.as<uint32_t>(),
                     (const uint32_t*)c->neg_g2.as<uint32_t>(), (const uint4*)R.pk_coeffs.as<uint4>(),
                     R.rec_f.as<uint4>(), R.rec_f2.as<uint4>(), M, d_group, (uint64_t)R.K, (const uint8_t*)nullptr);
  hipLaunchKernelGGL(k_fp12_prod_segs, dim3((unsigned)NR), dim3((unsigned)kProdLanes), 0, s, (uint32_t)NR, d_tbeg,
                     (const uint4*)R.rec_f.as<uint4>(), (uint64_t)M, R.part2.as<uint4>(), R.acc.as<uint4>());
  if (R.tmp.ensure(((NR + 63) / 64) * 8)) return CESS_BLS_E_OOM;
  r = rlc_final_exp(c, R, NR, s, gt_out != nullptr);
  if (r) return r;
  std::vector<uint8_t> codes(NR);
  HIPCHK(hipMemcpyAsync(codes.data(), R.fin_code.p, NR, hipMemcpyDeviceToHost, s));
  if (gt_out) HIPCHK(hipMemcpyAsync(gt_out, R.gt.p, 576, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  for (uint64_t q = 0; q < NR; q++) ok[q] = codes[q] == CODE_OK;
  return CESS_BLS_OK;
}

// ---- distinct-key RLC (CESS_BLS_F_RLC_DISTINCT) -------------------------------
// Scalars: r_i = a + b lambda with 32-bit a (odd), b from the record's
// rlc_scalar and lambda phi's eigenvalue on G1 (k_rlcd_scale,
// g1_mul_glv32): 2^63 values, so an invalid batch passes a check with
// probability <= 2^-63 (Ethereum consensus clients batch BLS with 64-bit
// exponents), for 32 doublings + 32 additions per point instead of the
// 128-bit form's 128 + 64.
// Ranges are record-index ranges [a, b) (R.perm is the identity) whose start
// and end (unless n) are multiples of kRlcdPer.  A range's check: S_r = sum of
// P_i = r_i sig_i (k_rlcd_scale; identity for records with a code),
// Miller(S_r, -G2), times the product of the range's stored lane values g_k =
// prod f_i over i in [kRlcdPer k, kRlcdPer (k + 1)), f_i = Miller(r_i H_i, pk_i)
// (k_miller_rr; one for records with a code), then one final exponentiation.  The products run in chunk passes (kRlcdChunk values per
// lane) until every range has at most 256 partials, then k_fp12_prod_segs.
constexpr uint64_t kRlcdChunk = 8;
constexpr uint64_t kRlcdPer = CESS_RLCD_PER;
// Part 1 of a check, on stream t: S_r = sum of the range's P_i and
// Miller(S_r, -G2) into R.rec_f2 (the batch's first check runs it on stream2,
// beside the last chunk's Miller loops: the single-wave S loop is latency).
static int rlcd_s_part(cess_bls_ctx* c, RlcState& R, const std::vector<std::pair<uint64_t, uint64_t>>& rg,
                       hipStream_t t) {
  const uint64_t NR = rg.size(), n = R.n;
  std::vector<uint64_t> so(NR), sc(NR);
  for (uint64_t q = 0; q < NR; q++) so[q] = rg[q].first, sc[q] = rg[q].second - rg[q].first;
  int r = R.S.ensure(NR * 36 * 4) | R.rec_code.ensure(NR) | R.rec_sig.ensure(NR * CESS_W_G1 * 4);
  r |= R.rec_f2.ensure(NR * CESS_W_FP12 * 4) | R.slots.ensure(NR * CESS_W_FP12 * 4 * CESS_FE_SLOTS);
  r |= R.fin_bm.ensure(NR);   // the S records' inf flags (k_rlcd_s_records)
  if (r) return CESS_BLS_E_OOM;
  r = rlc_sums(R, t, so, sc, R.P.as<uint32_t>(), n, R.S.as<uint32_t>(), NR);
  if (r) return r;
  hipLaunchKernelGGL(k_rlcd_s_records, dim3((unsigned)((NR + 63) / 64)), dim3(64), 0, t, (uint32_t)NR,
                     (const uint32_t*)R.S.as<uint32_t>(), R.rec_code.as<uint8_t>(), R.fin_bm.as<uint8_t>(),
                     R.rec_sig.as<uint32_t>());
  hipLaunchKernelGGL(k_miller, dim3(grid_for(NR)), dim3(kBlock), 0, t, NR, (const uint8_t*)R.rec_code.as<uint8_t>(),
                     (const uint8_t*)R.fin_bm.as<uint8_t>(), (const uint32_t*)R.rec_sig.as<uint32_t>(),
                     (const uint32_t*)R.rec_sig.as<uint32_t>(), (const uint32_t*)c->neg_g2.as<uint32_t>(),
                     (const uint4*)nullptr, R.rec_f2.as<uint4>(), R.slots.as<uint4>(), NR, (const uint32_t*)nullptr,
                     NR, (const uint8_t*)nullptr);
  HIPCHK(hipGetLastError());
  return CESS_BLS_OK;
}

// Part 2, on the context stream (after part 1: `wait`, an event of part 1's
// stream, or nullptr when part 1 ran on this stream): per-range products of
// the stored f_i in chunk passes (kRlcdChunk values per lane) until every
// range has at most 256 partials, then k_fp12_prod_segs, times Miller(S_r),
// and one final exponentiation per range: ok[r] = range r passes.
static int rlcd_final_part(cess_bls_ctx* c, RlcState& R, const std::vector<std::pair<uint64_t, uint64_t>>& rg,
                           hipEvent_t wait, std::vector<uint8_t>& ok, uint8_t* gt_out) {
  hipStream_t s = c->stream;
  const uint64_t NR = rg.size(), n = R.n;
  int r = R.acc.ensure(NR * CESS_W_FP12 * 4) | R.part2.ensure(NR * kProdLanes * CESS_W_FP12 * 4);
  r |= R.fin_code.ensure(NR) | R.gt.ensure(NR * 576) | R.tmp.ensure(((NR + 63) / 64) * 8);
  if (r) return CESS_BLS_E_OOM;
  std::vector<uint64_t> cnt(NR), base(NR);   // values per range in the current input, their first index
  for (uint64_t q = 0; q < NR; q++) {
    // record range [a, b) -> lane values [a / P, ceil(b / P))
    if (rg[q].first % kRlcdPer || (rg[q].second % kRlcdPer && rg[q].second != n) || rg[q].second < rg[q].first)
      return CESS_BLS_E_INVALID_ARG;
    base[q] = rg[q].first / kRlcdPer;
    cnt[q] = (rg[q].second + kRlcdPer - 1) / kRlcdPer - base[q];
  }
  const uint4* in = R.d_rec_f.as<uint4>();
  uint64_t in_stride = (n + kRlcdPer - 1) / kRlcdPer;
  const uint8_t* in_code = nullptr;
  bool flip = false;
  for (;;) {
    uint64_t mx = 0;
    for (uint64_t v : cnt) mx = std::max(mx, v);
    if (mx <= 4 * kProdLanes && in != R.d_rec_f.as<uint4>()) break;
    std::vector<uint64_t> lo, hi, nb(NR);
    for (uint64_t q = 0; q < NR; q++) {
      nb[q] = lo.size();
      for (uint64_t a = 0; a < cnt[q]; a += kRlcdChunk) {
        lo.push_back(base[q] + a);
        hi.push_back(base[q] + std::min(cnt[q], a + kRlcdChunk));
      }
      if (cnt[q] == 0) {   // an empty range still needs its (one) partial
        lo.push_back(base[q]);
        hi.push_back(base[q]);
      }
    }
    const uint64_t nch = lo.size();
    if (nch >= (1ull << 31)) return CESS_BLS_E_INVALID_ARG;
    DevBuf& out = flip ? R.pr_b : R.pr_a;
    if (out.ensure(nch * CESS_W_FP12 * 4) | R.pr_lo.ensure(nch * 8) | R.pr_hi.ensure(nch * 8)) return CESS_BLS_E_OOM;
    HIPCHK(hipMemcpyAsync(R.pr_lo.p, lo.data(), nch * 8, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(R.pr_hi.p, hi.data(), nch * 8, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_fp12_prod_chunks, dim3((unsigned)((nch + 255) / 256)), dim3(256), 0, s, (uint32_t)nch,
                       (const uint64_t*)R.pr_lo.as<uint64_t>(), (const uint64_t*)R.pr_hi.as<uint64_t>(), in_code, in,
                       in_stride, out.as<uint4>());
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(s));   // lo / hi are host vectors
    for (uint64_t q = 0; q < NR; q++) {
      base[q] = nb[q];
      cnt[q] = (q + 1 < NR ? nb[q + 1] : nch) - nb[q];
    }
    in = out.as<uint4>();
    in_stride = nch;
    in_code = nullptr;
    flip = !flip;
  }
  std::vector<uint32_t> tb(NR + 1);
  for (uint64_t q = 0; q < NR; q++) tb[q] = (uint32_t)base[q];
  tb[NR] = (uint32_t)(base[NR - 1] + cnt[NR - 1]);
  if (R.lists.ensure((NR + 1) * 4)) return CESS_BLS_E_OOM;
  HIPCHK(hipMemcpyAsync(R.lists.p, tb.data(), (NR + 1) * 4, hipMemcpyHostToDevice, s));
  hipLaunchKernelGGL(k_fp12_prod_segs, dim3((unsigned)NR), dim3((unsigned)kProdLanes), 0, s, (uint32_t)NR,
                     (const uint32_t*)R.lists.as<uint32_t>(), in, in_stride, R.part2.as<uint4>(), R.acc.as<uint4>());
  if (wait) HIPCHK(hipStreamWaitEvent(s, wait, 0));
  hipLaunchKernelGGL(k_fp12_mul_each, dim3((unsigned)((NR + 63) / 64)), dim3(64), 0, s, (uint32_t)NR,
                     R.acc.as<uint4>(), (const uint4*)R.rec_f2.as<uint4>());
  r = rlc_final_exp(c, R, NR, s, gt_out != nullptr);
  if (r) return r;
  std::vector<uint8_t> codes(NR);
  HIPCHK(hipMemcpyAsync(codes.data(), R.fin_code.p, NR, hipMemcpyDeviceToHost, s));
  if (gt_out) HIPCHK(hipMemcpyAsync(gt_out, R.gt.p, 576, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));   // tb is a host vector
  ok.assign(NR, 1);
  for (uint64_t q = 0; q < NR; q++) ok[q] = codes[q] == CODE_OK;
  return CESS_BLS_OK;
}

// A check of the record ranges rg (both parts on the context stream).
static int rlcd_check(cess_bls_ctx* c, RlcState& R, const std::vector<std::pair<uint64_t, uint64_t>>& rg,
                      std::vector<uint8_t>& ok, uint8_t* gt_out) {
  const uint64_t NR = rg.size();
  R.checks += NR;
  ok.assign(NR, 1);
  if (NR == 0) return CESS_BLS_OK;
  if (NR >= (1ull << 31)) return CESS_BLS_E_INVALID_ARG;
  int r = rlcd_s_part(c, R, rg, c->stream);
  if (r) return r;
  return rlcd_final_part(c, R, rg, nullptr, ok, gt_out);
}

// The batch's records through the per-signature light kernels in chunks of
// qcap, then P_i, Q_i (k_rlcd_scale) and f_i = Miller(Q_i, pk_i) kept for the
// whole batch; then the batch check.
static int rlcd_begin(cess_bls_ctx* c, RlcState& R, const uint8_t* seed32, uint64_t index_hi, uint8_t* gt_out) {
  hipStream_t s = c->stream;
  const uint64_t n = R.n, q = c->qcap;
  R.distinct = true;
  R.K = 0;
  R.perm.resize(n);
  for (uint64_t i = 0; i < n; i++) R.perm[i] = (uint32_t)i;
  int r = R.P.ensure(n * 36 * 4) | R.Q.ensure(n * 36 * 4) | R.d_code.ensure(n) | R.d_perm.ensure(n * 4);
  r |= R.d_rec_f.ensure(((n + kRlcdPer - 1) / kRlcdPer) * CESS_W_FP12 * 4) | R.d_seed.ensure(32) | R.rec_h.ensure(q * CESS_W_G1 * 4);
  r |= R.rec_inf.ensure(q);
  StageSlot& S = c->slot[0];
  r |= S.inf.ensure(q) | S.sig_aff.ensure(q * CESS_W_G1 * 4) | S.h_aff.ensure(q * CESS_W_G1 * 4) |
       S.pk_aff.ensure(q * CESS_W_G2 * 4) | S.coeffs.ensure(q * (uint64_t)CESS_W_COEFFS * 4);
  if (r) return CESS_BLS_E_OOM;
  {
    uint32_t sw[8];
    for (int w = 0; w < 8; w++)
      sw[w] = ((uint32_t)seed32[4 * w] << 24) | ((uint32_t)seed32[4 * w + 1] << 16) | ((uint32_t)seed32[4 * w + 2] << 8) |
              seed32[4 * w + 3];
    HIPCHK(hipMemcpyAsync(R.d_seed.p, sw, 32, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(R.d_perm.p, R.perm.data(), n * 4, hipMemcpyHostToDevice, s));
    HIPCHK(hipStreamSynchronize(s));   // sw is a stack buffer
  }
  const uint32_t strict = (c->flags & CESS_BLS_F_STRICT_IDENTITY) ? 1u : 0u;
  std::vector<uint64_t> rebased;
  // chunks start at multiples of kRlcdPer (k_miller_rr's lanes)
  const uint64_t step = q >= kRlcdPer ? q - q % kRlcdPer : q;
  for (uint64_t off = 0; off < n; off += step) {
    const uint64_t m = std::min<uint64_t>(step, n - off);
    const uint64_t mb0 = R.offs[off], mb1 = R.offs[off + m];
    if (mb1 < mb0) return CESS_BLS_E_INVALID_ARG;
    rebased.resize(m + 1);
    for (uint64_t j = 0; j <= m; j++) {
      if (j && R.offs[off + j] < R.offs[off + j - 1]) return CESS_BLS_E_INVALID_ARG;
      rebased[j] = R.offs[off + j] - mb0;
    }
    r = c->in_sigs.ensure(m * 48) | c->in_pks.ensure(m * 96) | c->in_msgs.ensure(std::max<uint64_t>(mb1 - mb0, 1)) |
        c->in_offs.ensure((m + 1) * 8);
    if (r) return CESS_BLS_E_OOM;
    HIPCHK(hipMemcpyAsync(c->in_sigs.p, R.sigs + 48 * off, m * 48, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(c->in_pks.p, R.pks + 96 * off, m * 96, hipMemcpyHostToDevice, s));
    if (mb1 > mb0) HIPCHK(hipMemcpyAsync(c->in_msgs.p, R.msgs + mb0, mb1 - mb0, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(c->in_offs.p, rebased.data(), (m + 1) * 8, hipMemcpyHostToDevice, s));
    uint8_t* code = R.d_code.as<uint8_t>() + off;
    uint8_t* inf = S.inf.as<uint8_t>();
    HIPCHK(hipMemsetAsync(code, 0, m, s));
    HIPCHK(hipMemsetAsync(inf, 0, m, s));
    const unsigned g = grid_for(m);
    // the per-signature decode / hash / prepare (run_chunk's light kernels;
    // codes in the reference's precedence)
    RLAUNCH(ST_DECODE_SIG, s, k_decode_sig, dim3(g), dim3(kBlock), 0, s, m, c->in_sigs.as<uint8_t>(), (const uint8_t*)nullptr,
                       code, inf, S.sig_aff.as<uint32_t>(), q);
    RLAUNCH(ST_DECODE_PK, s, k_decode_pk, dim3(g), dim3(kBlock), 0, s, m, c->in_pks.as<uint8_t>(), (const uint8_t*)nullptr,
                       code, inf, S.pk_aff.as<uint32_t>(), q, strict);
    RLAUNCH(ST_HASH, s, k_hash, dim3(g), dim3(kBlock), 0, s, m, c->in_msgs.as<uint8_t>(), c->in_offs.as<uint64_t>(),
                       (const uint8_t*)code, S.h_aff.as<uint32_t>(), q);
    RLAUNCH(ST_PREPARE, s, k_prepare, dim3(g), dim3(kBlock), 0, s, m, (const uint32_t*)S.pk_aff.as<uint32_t>(),
                       S.coeffs.as<uint4>(), q, code, (const uint8_t*)inf);
    // P_i = r_i sig_i, Q_i = r_i H_i (stride n), then f_i = Miller(Q_i, pk_i)
    hipLaunchKernelGGL(k_rlcd_scale, dim3(g), dim3(kBlock), 0, s, m, (const uint8_t*)code, (const uint8_t*)inf,
                       (const uint32_t*)S.sig_aff.as<uint32_t>(), (const uint32_t*)S.h_aff.as<uint32_t>(),
                       (const uint32_t*)R.d_seed.as<uint32_t>(), index_hi + off, R.P.as<uint32_t>() + off,
                       R.Q.as<uint32_t>() + off, q, n);
    // the last chunk: every P_i exists once this k_rlcd_scale is done
    const bool last = off + m == n;
    if (last) HIPCHK(hipEventRecord(c->ev_start, s));
    hipLaunchKernelGGL(k_rlcd_records, dim3(g), dim3(kBlock), 0, s, m, (const uint8_t*)code, (const uint8_t*)inf,
                       (const uint32_t*)(R.Q.as<uint32_t>() + off), n, R.rec_h.as<uint32_t>(), R.rec_inf.as<uint8_t>(),
                       q);
    // g_k straight into the batch-wide lane values (stride ceil(n / P))
    const uint64_t np = (m + kRlcdPer - 1) / kRlcdPer;
    // (k_miller_rr2: a lane pair per lane of records, two waves per SIMD,
    // unless CESS_BLS_MILLER=lane selects the one-lane kernels)
    static const bool rr_pair = !(getenv("CESS_BLS_MILLER") && strcmp(getenv("CESS_BLS_MILLER"), "lane") == 0);
    RLAUNCH(ST_MILLER, s, rr_pair ? k_miller_rr2 : k_miller_rr,
            dim3(rr_pair ? (unsigned)((np + CESS_PAIR_THREADS / 2 - 1) / (CESS_PAIR_THREADS / 2)) : grid_for(np)),
            dim3(rr_pair ? CESS_PAIR_THREADS : kBlock), 0, s, np, m, (const uint8_t*)code,
                       (const uint8_t*)R.rec_inf.as<uint8_t>(), (const uint32_t*)R.rec_h.as<uint32_t>(),
                       (const uint4*)S.coeffs.as<uint4>(), R.d_rec_f.as<uint4>() + off / kRlcdPer, q,
                       (n + kRlcdPer - 1) / kRlcdPer);
    HIPCHK(hipGetLastError());
    if (last) {
      // the batch's S sum and its single-wave Miller loop on stream2, after
      // this chunk's k_rlcd_scale (ev_start): this chunk's k_rlcd_records and
      // k_miller_rr are already enqueued on s, so they run beside it even
      // though rlc_sums blocks the host until its segment table is consumed
      HIPCHK(hipStreamWaitEvent(c->stream2, c->ev_start, 0));
      R.checks += 1;
      r = rlcd_s_part(c, R, {{0, n}}, c->stream2);
      if (r) return r;
      HIPCHK(hipEventRecord(c->ev_light[0], c->stream2));
    }
    HIPCHK(hipMemcpyAsync(&R.codes[off], code, m, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));   // rebased is reused by the next chunk
  }
  std::vector<uint8_t> ok;
  r = rlcd_final_part(c, R, {{0, n}}, c->ev_light[0], ok, gt_out);
  if (r) return r;
  R.local_ok = ok[0] != 0;
  return CESS_BLS_OK;
}

// rlc_begin with an index base for the scalars (ranks pass rank << 40, so no
// r_i is shared across shards under one seed)
int cess_host::rlc_begin_at(cess_bls_ctx* c, size_t n, const uint8_t* sigs, const uint8_t* pks, const uint8_t* msgs,
                        const uint64_t* offs, const uint8_t* seed_in, uint64_t index_hi, uint8_t* gt_out) {
  if (c->rlc) c->rlc->valid = false;   // whatever happens below, the previous batch is gone
  if (n && (!sigs || !pks || !offs || (!msgs && offs[n] != offs[0]))) return CESS_BLS_E_INVALID_ARG;
  if (n >= (1ull << 32)) return CESS_BLS_E_INVALID_ARG;
  uint8_t seed32[32];
  if (seed_in) memcpy(seed32, seed_in, 32);
  else if (os_random(seed32, 32)) return CESS_BLS_E_INVALID_ARG;
  HIPCHK(hipSetDevice(c->device));
  if (!c->rlc) c->rlc = new RlcState();
  RlcState& R = *c->rlc;
  R.n = n, R.sigs = sigs, R.pks = pks, R.msgs = msgs, R.offs = offs;
  R.checks = R.leaves = R.leaf_sigs = 0;
  R.codes.assign(n, 0);
  R.local_ok = false;
  R.valid = false;
  R.per_sig = false;
  R.K = 0;
  R.pts = R.pq = R.aos = R.have_pos = false;
  R.distinct = false;
  R.index_hi = index_hi;
  auto gt_one = [&]() {
    if (gt_out) {   // the empty product: Gt one
      memset(gt_out, 0, 576);
      gt_out[47] = 1;
    }
  };
  if (n == 0) {
    gt_one();
    R.local_ok = R.valid = true;
    return CESS_BLS_OK;
  }
  hipStream_t s = c->stream;
  int r = order_begin(c, s);
  if (r) return r;
  if (c->flags & CESS_BLS_F_RLC_DISTINCT) {
    r = rlcd_begin(c, R, seed32, index_hi, gt_out);
    if (r) return r;
    r = order_end(c, s);
    if (r) return r;
    R.valid = true;
    return CESS_BLS_OK;
  }
  // 1. key groups (dedup of the 96-byte encodings; open addressing on a
  //    64-bit hash, full compare) and a counting sort by group.  Slices of the
  //    batch are deduplicated on host threads, then their distinct keys are
  //    merged in slice order, so group ids follow first occurrence exactly as
  //    a sequential pass would number them.
  std::vector<uint32_t> grp(n);
  std::vector<uint64_t> first;
  group_keys(pks, n, grp, first);
  const uint32_t K = R.K = (uint32_t)first.size();
  // 1b. many distinct keys: a combination needs K + 1 pairings anyway and a
  //     forgery's bisection would cost more than per-signature verification,
  //     so the shard is verified per signature (exact codes, Gt partial one)
  if (8 * (uint64_t)K > n) {
    R.per_sig = true;
    r = verify_host(c, n, sigs, pks, msgs, offs, nullptr, R.codes.data(), nullptr, nullptr);
    if (r) return r;
    R.leaf_sigs = n;
    gt_one();
    R.valid = true;
    return CESS_BLS_OK;
  }
  R.gbeg.assign(K + 1, 0);
  for (uint64_t i = 0; i < n; i++) R.gbeg[grp[i] + 1]++;
  for (uint32_t g = 0; g < K; g++) R.gbeg[g + 1] += R.gbeg[g];
  R.perm.resize(n);
  {
    std::vector<uint64_t> pos(R.gbeg.begin(), R.gbeg.end() - 1);
    for (uint64_t i = 0; i < n; i++) R.perm[pos[grp[i]]++] = (uint32_t)i;
  }
  // 2. device buffers (bucket path: the batch's points and codes stay on the
  //    device for msm_sums; per-record multiples only if bisection needs them)
  R.pts = msm_ok(n, (uint64_t)K + 1);
  R.pq = !R.pts;
  r = 0;
  if (R.pts) {
    r |= R.Xs.ensure(n * CESS_W_G1 * 4) | R.Xh.ensure(n * CESS_W_G1 * 4) | R.d_code.ensure(n) | R.d_inf.ensure(n);
    r |= R.d_grp.ensure(n * 4);
  } else {
    r |= R.P.ensure(n * 36 * 4) | R.Q.ensure(n * 36 * 4);
  }
  r |= R.d_perm.ensure(n * 4) | R.d_seed.ensure(32);
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
    HIPCHK(hipStreamSynchronize(s));   // sw is a stack buffer
  }
  HIPCHK(hipMemcpyAsync(R.d_perm.p, R.perm.data(), n * 4, hipMemcpyHostToDevice, s));
  if (R.pts) HIPCHK(hipMemcpyAsync(R.d_grp.p, grp.data(), n * 4, hipMemcpyHostToDevice, s));
  // 3. distinct keys: decode (G2Affine::from_compressed, src/lib.rs:74) + G2Prepared (:88), once per key
  std::vector<uint8_t> kbytes((uint64_t)K * 96), pkc(K), pki(K), usable(K);
  for (uint32_t g = 0; g < K; g++) memcpy(&kbytes[96 * (uint64_t)g], pks + 96 * first[g], 96);
  const uint32_t strict = (c->flags & CESS_BLS_F_STRICT_IDENTITY) ? 1u : 0u;
  HIPCHK(hipMemcpyAsync(R.pk_in.p, kbytes.data(), kbytes.size(), hipMemcpyHostToDevice, s));
  HIPCHK(hipMemsetAsync(R.pk_code.p, 0, K, s));
  HIPCHK(hipMemsetAsync(R.pk_inf.p, 0, K, s));
  hipLaunchKernelGGL(k_decode_pk, dim3(grid_for(K)), dim3(kBlock), 0, s, (uint64_t)K, R.pk_in.as<uint8_t>(),
                     (const uint8_t*)nullptr, R.pk_code.as<uint8_t>(), R.pk_inf.as<uint8_t>(), R.pk_aff.as<uint32_t>(),
                     (uint64_t)K, strict);
  hipLaunchKernelGGL(k_prepare, dim3(grid_for(K)), dim3(kBlock), 0, s, (uint64_t)K,
                     (const uint32_t*)R.pk_aff.as<uint32_t>(), R.pk_coeffs.as<uint4>(), (uint64_t)K,
                     R.pk_code.as<uint8_t>(), (const uint8_t*)R.pk_inf.as<uint8_t>());
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
  for (uint64_t off = 0; off < n; off += c->qcap) {
    const uint64_t m = std::min<uint64_t>(c->qcap, n - off);
    const uint64_t mb0 = offs[off], mb1 = offs[off + m];
    if (mb1 < mb0) return CESS_BLS_E_INVALID_ARG;
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
    StageSlot& S = c->slot[0];
    // the points go to the batch-wide arrays (stride n) on the bucket path
    uint32_t* sig_dst = R.pts ? R.Xs.as<uint32_t>() + off : S.sig_aff.as<uint32_t>();
    uint32_t* h_dst = R.pts ? R.Xh.as<uint32_t>() + off : S.h_aff.as<uint32_t>();
    const uint64_t pstride = R.pts ? n : c->qcap;
    RLAUNCH(ST_DECODE_SIG, s, k_decode_sig, dim3(g), dim3(kBlock), 0, s, m, c->in_sigs.as<uint8_t>(), (const uint8_t*)nullptr,
                       c->code.as<uint8_t>(), S.inf.as<uint8_t>(), sig_dst, pstride);
    HIPCHK(hipGetLastError());
    hc.resize(m);
    hi.resize(m);
    HIPCHK(hipMemcpyAsync(hc.data(), c->code.p, m, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(hi.data(), S.inf.p, m, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    for (uint64_t j = 0; j < m; j++) {
      if (hc[j] != 0) continue;
      const uint32_t gg = grp[off + j];
      if (pkc[gg] != 0) hc[j] = pkc[gg];
      else if (pki[gg] & INF_PK) hi[j] |= INF_PK;
    }
    memcpy(&R.codes[off], hc.data(), m);
    HIPCHK(hipMemcpyAsync(c->code.p, hc.data(), m, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(S.inf.p, hi.data(), m, hipMemcpyHostToDevice, s));
    RLAUNCH(ST_HASH, s, k_hash, dim3(g), dim3(kBlock), 0, s, m, c->in_msgs.as<uint8_t>(), c->in_offs.as<uint64_t>(),
                       (const uint8_t*)c->code.as<uint8_t>(), h_dst, pstride);
    if (R.pts) {
      HIPCHK(hipMemcpyAsync(R.d_code.as<uint8_t>() + off, hc.data(), m, hipMemcpyHostToDevice, s));
      HIPCHK(hipMemcpyAsync(R.d_inf.as<uint8_t>() + off, hi.data(), m, hipMemcpyHostToDevice, s));
    } else {
      hipLaunchKernelGGL(k_rlc_scale, dim3(g), dim3(kBlock), 0, s, m, (const uint8_t*)c->code.as<uint8_t>(),
                         (const uint8_t*)S.inf.as<uint8_t>(), (const uint32_t*)S.sig_aff.as<uint32_t>(),
                         (const uint32_t*)S.h_aff.as<uint32_t>(), (const uint32_t*)R.d_seed.as<uint32_t>(),
                         index_hi + off, R.P.as<uint32_t>() + off, R.Q.as<uint32_t>() + off, c->qcap, (uint64_t)n, 4u);
    }
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(s));   // hc/hi are reused by the next chunk
  }
  // 5. the batch check (this shard's Gt partial)
  std::vector<uint8_t> ok;
  r = rlc_check_multi(c, R, {{0, n}}, ok, gt_out);
  if (r) return r;
  R.local_ok = ok[0] != 0;
  r = order_end(c, s);
  if (r) return r;
  R.valid = true;
  return CESS_BLS_OK;
}

int cess_host::rlc_begin(cess_bls_ctx* c, size_t n, const uint8_t* sigs, const uint8_t* pks, const uint8_t* msgs,
                         const uint64_t* offs, const uint8_t* seed32, uint8_t* gt_out) {
  const uint64_t hi = c->xport ? ((uint64_t)c->rank << 40) : 0;
  return rlc_begin_at(c, n, sigs, pks, msgs, offs, seed32, hi, gt_out);
}

int cess_host::gt_product_is_one(cess_bls_ctx* c, size_t m, const uint8_t* gts, bool on_device, int* is_one) {
  HIPCHK(hipSetDevice(c->device));
  if (!c->rlc) c->rlc = new RlcState();
  RlcState& R = *c->rlc;
  if (m == 0) {
    *is_one = 1;
    return CESS_BLS_OK;
  }
  hipStream_t s = c->stream;
  int r = order_begin(c, s);
  if (r) return r;
  if (R.gts.ensure(m * 576) | R.tmp.ensure(2 * CESS_W_FP12 * 4) | R.fin_code.ensure(1)) return CESS_BLS_E_OOM;
  const uint8_t* d_gts = gts;
  if (!on_device) {
    HIPCHK(hipMemcpyAsync(R.gts.p, gts, m * 576, hipMemcpyHostToDevice, s));
    d_gts = R.gts.as<uint8_t>();
  }
  hipLaunchKernelGGL(k_gt_prod, dim3(1), dim3(64), 0, s, (uint32_t)m, d_gts, R.tmp.as<uint4>(), R.fin_code.as<uint8_t>());
  HIPCHK(hipGetLastError());
  uint8_t code = 0xff;
  HIPCHK(hipMemcpyAsync(&code, R.fin_code.p, 1, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  *is_one = code == CODE_OK;
  return order_end(c, s);
}

// Bisect iff this shard's own check failed: honest records contribute exactly
// one to the shard's partial, so a failed local check proves an invalid member,
// and no other shard's partial may cancel that proof.
int cess_host::rlc_finish(cess_bls_ctx* c, uint8_t* codes_out, uint64_t* bitmap_out, uint64_t* stats4) {
  if (!c->rlc || !c->rlc->valid) return CESS_BLS_E_INVALID_ARG;
  RlcState& R = *c->rlc;
  R.valid = false;   // one finish per begin; a failure below leaves nothing to finish
  const uint64_t n = R.n;
  std::vector<uint8_t>& codes = R.codes;
  if (!R.per_sig && !R.local_ok) {
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
        const uint64_t fan = std::min<uint64_t>(R.distinct ? kRlcdFan : kRlcFan, (len + kRlcLeaf - 1) / kRlcLeaf);
        // distinct-key ranges split at multiples of kRlcdPer (the stored
        // values are per lane); a part keeps > kRlcLeaf / 2 records
        const uint64_t al = R.distinct ? kRlcdPer : 1;
        auto cut = [&](uint64_t q) { return q == fan ? w.second : w.first + (len * q / fan) / al * al; };
        for (uint64_t q = 0; q < fan; q++) parts.push_back({cut(q), cut(q + 1)});
      }
      level.clear();
      if (!parts.empty()) {
        int r = R.distinct ? rlcd_check(c, R, parts, ok, nullptr) : rlc_check_multi(c, R, parts, ok, nullptr);
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
  if (bitmap_out) bitmap_from_codes(codes.data(), n, bitmap_out);
  if (stats4) {
    stats4[0] = R.checks;
    stats4[1] = R.leaves;
    stats4[2] = R.leaf_sigs;
    stats4[3] = R.K;
  }
  return CESS_BLS_OK;
}

int cess_host::verify_rlc_host(cess_bls_ctx* c, size_t n, const uint8_t* sigs, const uint8_t* pks, const uint8_t* msgs,
                               const uint64_t* offs, const uint8_t* seed32, uint8_t* codes_out, uint64_t* bitmap_out,
                               uint64_t* stats4) {
  int r = rlc_begin_at(c, n, sigs, pks, msgs, offs, seed32, 0, nullptr);
  if (r) return r;
  r = rlc_finish(c, codes_out, bitmap_out, stats4);
  if (r) return r;
  return collect_profile(c, c->stream);   // no-op without CESS_BLS_F_PROFILE
}

#define ENTRY(c)                          \
  if (!(c)) return CESS_BLS_E_INVALID_ARG; \
  CtxLock lock_(c);                        \
  if (!lock_.ok()) return CESS_BLS_E_BUSY

int cess_multi_verify(cess_bls_ctx* c, size_t n, const uint8_t* sigs, const uint8_t* pks, const uint8_t* msgs,
                      const uint64_t* offs, uint8_t* codes_out, uint64_t* bitmap_out, bool rlc, const uint8_t* seed32,
                      uint64_t* stats4);

extern "C" int cess_bls_rlc_begin(cess_bls_ctx* c, size_t n, const uint8_t* sigs, const uint8_t* pks,
                                  const uint8_t* msgs, const uint64_t* offs, const uint8_t* seed32, uint8_t* gt_out) {
  ENTRY(c);
  if (!c->subs.empty()) return CESS_BLS_E_INVALID_ARG;
  return rlc_begin(c, n, sigs, pks, msgs, offs, seed32, gt_out);
}

extern "C" int cess_bls_gt_product_is_one(cess_bls_ctx* c, size_t m, const uint8_t* gts, int* is_one) {
  ENTRY(c);
  if (!is_one || (m && !gts)) return CESS_BLS_E_INVALID_ARG;
  cess_bls_ctx* d = c->subs.empty() ? c : c->subs[0];
  return gt_product_is_one(d, m, gts, false, is_one);
}

extern "C" int cess_bls_rlc_finish(cess_bls_ctx* c, int global_ok, uint8_t* codes_out, uint64_t* bitmap_out,
                                   uint64_t* stats4) {
  ENTRY(c);
  (void)global_ok;   // a batch-level summary only; see rlc_finish
  if (!c->subs.empty()) return CESS_BLS_E_INVALID_ARG;
  return rlc_finish(c, codes_out, bitmap_out, stats4);
}

extern "C" int cess_bls_verify_batch_rlc(cess_bls_ctx* c, size_t n, const uint8_t* sigs, const uint8_t* pks,
                                         const uint8_t* msgs, const uint64_t* msg_offsets, const uint8_t* seed32,
                                         uint8_t* codes_out, uint64_t* bitmap_out, uint64_t* stats4) {
  ENTRY(c);
  if (!c->subs.empty())
    return cess_multi_verify(c, n, sigs, pks, msgs, msg_offsets, codes_out, bitmap_out, true, seed32, stats4);
  return verify_rlc_host(c, n, sigs, pks, msgs, msg_offsets, seed32, codes_out, bitmap_out, stats4);
}
