// CDNA4 (gfx950) kernels of the random-linear-combination (RLC) batch mode
// (BASELINE north_star "optional random-linear-combination batch mode"; SURVEY
// §8(d) C4 / §8(e)).  For a (sub)batch with distinct keys pk_1..pk_K:
//
//   e(sum_i r_i sig_i, -G2) * prod_k e(sum_{i: pk_i = pk_k} r_i H(m_i), pk_k) == 1
//
// holds iff every member passes verify_bls_signature's pairing equation
// (src/lib.rs:85-100), except with probability <= 2^-127 over the 128-bit r_i.
// Malformed encodings never enter the sums: they keep their decode codes.
//
// k_msm_*      : the sums of a check by buckets (Pippenger), the default path
// k_rlc_scale  : P_i = r_i sig_i, Q_i = r_i H(m_i)   (r_i = SHA-256(seed || i)[0:16] | 1),
//                for checks with too many segments for the bucket tables
// k_g1_sum_segs    : segmented sums of projective G1 points over permuted index ranges
// k_rlc_pairs_list : (range, key group) terms -> affine Miller-loop records (k_miller input)
// k_fp12_prod_segs : per-range product of the terms' Miller-loop values
// k_gt_prod        : product of m canonical Gt values == 1 ?  (cross-rank combine)
#include <hip/hip_runtime.h>
#include "soa.hpp"

using namespace bls;
using namespace cess;

namespace {

// projective G1 in SoA: x at words 0..11, y 12..23, z 24..35
__device__ __forceinline__ g1p ld_g1p(const uint32_t* b, uint64_t stride, uint32_t i) {
  return {ld_fp(b, stride, i), ld_fp(b + 12 * stride, stride, i), ld_fp(b + 24 * stride, stride, i)};
}
__device__ __forceinline__ void st_g1p(uint32_t* b, uint64_t stride, uint32_t i, const g1p& p) {
  st_fp(b, stride, i, p.x);
  st_fp(b + 12 * stride, stride, i, p.y);
  st_fp(b + 24 * stride, stride, i, p.z);
}

// 128-bit scalar of record i from the batch seed (8 big-endian words)
__device__ void rlc_scalar(const uint32_t* seed, uint64_t i, uint32_t (&k)[4]) {
  uint32_t blk[16], st[8];
#pragma unroll
  for (int w = 0; w < 8; w++) blk[w] = seed[w], st[w] = SHA_IV[w];
  blk[8] = (uint32_t)(i >> 32);
  blk[9] = (uint32_t)i;
  blk[10] = 0x80000000u;
#pragma unroll
  for (int w = 11; w < 15; w++) blk[w] = 0;
  blk[15] = 320;   // 40-byte message
  sha256_compress(st, blk);
#pragma unroll
  for (int w = 0; w < 4; w++) k[w] = st[w];
  k[0] |= 1u;      // nonzero
}

}  // namespace

// [k]P for a 128-bit k and affine P (not the identity): 2-bit fixed windows with
// the table {P, 2P, 3P}; the window digit differs per lane, so the addition is
// computed every window and kept by a select (no divergent branches): 128
// doublings + 64 complete additions (a per-bit ladder costs 128 + 128 here,
// since some lane of the wave always takes the add).
// Force-inlined on purpose.  Round 1 saw the out-of-line (__noinline__) form
// hang; tools/rlc_call_probe.hip reproduces it and the ISA shows the cause: the
// callee body is longer than s_branch's +-2^15-dword reach, so branch
// relaxation expands long branches as s_getpc/s_add/s_setpc through s[30:31]
// -- the return-address pair of the AMDGPU call ABI -- without saving it.  The
// loop exit jumps to the return block through s[30:31] = &return block, and
// the return's s_setpc_b64 s[30:31] then spins on itself forever.  A compiler
// (branch-relaxation scavenging) defect, not a data race: the product library
// therefore contains no device calls at all (tests/test_isa_guard.py checks
// the shipped code objects for s_swappc_b64).
// (kwords = 4: the 128-bit scalar; 2: its low 64 bits -- the distinct-key
// mode's scalars, 32 windows instead of 64)
__device__ __forceinline__ g1p mul128_w2(const fp& px, const fp& py, const uint32_t (&k)[4], int kwords = 4) {
  const g1p T1 = {px, py, fp_one()};
  const g1p T2 = proj_dbl(T1);
  const g1p T3 = proj_add_mixed(T2, px, py);
  g1p acc = proj_identity<fp>();
#pragma unroll 1
  for (int w = kwords - 1; w >= 0; w--) {
#pragma unroll 1
    for (int b = 30; b >= 0; b -= 2) {
      acc = proj_dbl(proj_dbl(acc));
      const uint32_t d = (k[w] >> b) & 3u;
      const g1p t = {select(d == 1, T1.x, select(d == 2, T2.x, T3.x)), select(d == 1, T1.y, select(d == 2, T2.y, T3.y)),
                     select(d == 1, T1.z, select(d == 2, T2.z, T3.z))};
      const g1p sum = proj_add(acc, t);
      acc = {select(d != 0, sum.x, acc.x), select(d != 0, sum.y, acc.y), select(d != 0, sum.z, acc.z)};
    }
  }
  return acc;
}

// mul_glv32: curve.hpp g1_mul_glv32 (the distinct-key RLC's multiples)

// P_i = r_i sig_i, Q_i = r_i H_i (identity for records with a code or an
// identity point).  KW = 1: r_i = a + b lambda, a = k[0] | 1, b = k[1]
// (g1_mul_glv32); KW = 0: the 64-bit (kwords 2) or 128-bit (kwords 4) scalar
// (mul128_w2).  The distinct-key mode's KW = 1 is its own kernel
// (k_rlcd_scale), so its register allocation is not that of the 128-bit ladder.
template <int KW>
__device__ __forceinline__ void rlc_scale(uint64_t n, const uint8_t* __restrict__ code, const uint8_t* __restrict__ inf,
                                          const uint32_t* __restrict__ sig_aff, const uint32_t* __restrict__ h_aff,
                                          const uint32_t* __restrict__ seed, uint64_t index_base,
                                          uint32_t* __restrict__ P, uint32_t* __restrict__ Q, uint64_t stride,
                                          uint64_t out_stride, uint32_t kwords) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  g1p p = proj_identity<fp>(), q = proj_identity<fp>();
  const uint8_t fl = inf[i];
  if (code[i] == 0) {
    uint32_t k[4];
    rlc_scalar(seed, index_base + i, k);
    if constexpr (KW == 1) {
      const uint32_t a = k[0] | 1u, b = k[1];
      if ((fl & INF_SIG) == 0) p = g1_mul_glv32(ld_fp(sig_aff, stride, i), ld_fp(sig_aff + 12 * stride, stride, i), a, b);
      if ((fl & INF_PK) == 0) q = g1_mul_glv32(ld_fp(h_aff, stride, i), ld_fp(h_aff + 12 * stride, stride, i), a, b);
    } else {
      const int kw = kwords == 2 ? 2 : 4;
      if (kw == 2) k[2] = k[3] = 0;
      if ((fl & INF_SIG) == 0) p = mul128_w2(ld_fp(sig_aff, stride, i), ld_fp(sig_aff + 12 * stride, stride, i), k, kw);
      if ((fl & INF_PK) == 0) q = mul128_w2(ld_fp(h_aff, stride, i), ld_fp(h_aff + 12 * stride, stride, i), k, kw);
    }
  }
  st_g1p(P, out_stride, i, p);
  st_g1p(Q, out_stride, i, q);
}

// kwords 2 or 4 (see rlc_scale)
__global__ CESS_LB void k_rlc_scale(uint64_t n, const uint8_t* __restrict__ code, const uint8_t* __restrict__ inf,
                                    const uint32_t* __restrict__ sig_aff, const uint32_t* __restrict__ h_aff,
                                    const uint32_t* __restrict__ seed, uint64_t index_base, uint32_t* __restrict__ P,
                                    uint32_t* __restrict__ Q, uint64_t stride, uint64_t out_stride, uint32_t kwords) {
  rlc_scale<0>(n, code, inf, sig_aff, h_aff, seed, index_base, P, Q, stride, out_stride, kwords);
}

// the distinct-key mode's multiples (g1_mul_glv32)
#if defined(CESS_RLCD_SCALE_W1)   // one wave per SIMD: 512 registers, no scratch (sweep)
#define CESS_RLCD_SCALE_LB __launch_bounds__(256, 1)
#else
#define CESS_RLCD_SCALE_LB CESS_LB
#endif
__global__ CESS_RLCD_SCALE_LB void k_rlcd_scale(uint64_t n, const uint8_t* __restrict__ code, const uint8_t* __restrict__ inf,
                                     const uint32_t* __restrict__ sig_aff, const uint32_t* __restrict__ h_aff,
                                     const uint32_t* __restrict__ seed, uint64_t index_base, uint32_t* __restrict__ P,
                                     uint32_t* __restrict__ Q, uint64_t stride, uint64_t out_stride) {
  rlc_scale<1>(n, code, inf, sig_aff, h_aff, seed, index_base, P, Q, stride, out_stride, 1u);
}

// ---- bucket (Pippenger) sums of a check --------------------------------------
// A check needs only its segments' sums -- the batch's first check K + 1 of
// them: sum_i r_i sig_i and, per key group g, sum_{i in g} r_i H(m_i) -- so
// instead of one 128-bit scalar multiple per point (k_rlc_scale: 128
// doublings + 64 additions) the scalars are cut into 16 windows of 8 bits and
// each point is ADDED into one bucket per non-zero window digit: bucket b =
// (seg * 16 + w) * 256 + d (MsmSegs: which segments a record's signature and
// hash belong to).  Then W(seg, w) = sum_d d B(seg, w, d) (running sums), and
// S(seg) = sum_w 2^(8w) W(seg, w).  About 16 mixed additions per point instead
// of ~190 point operations (k_rlc_scale: 63 ms per 1 M records).  The sums
// are the same group elements, so every check and its Gt value are unchanged.
constexpr uint32_t MSM_WIN = 16, MSM_DIG = 256, MSM_SEG = MSM_WIN * MSM_DIG;

__device__ __forceinline__ uint32_t msm_digit(const uint32_t (&k)[4], uint32_t w) {
  return (k[w >> 2] >> (8 * (w & 3))) & 255u;   // k[0] is the least significant word
}

// index of the range [lo[a], hi[a]) holding position p, or -1 (lo sorted)
__device__ __forceinline__ int msm_find(const uint32_t* __restrict__ lo, const uint32_t* __restrict__ hi, uint32_t cnt,
                                        uint32_t p) {
  if (cnt == 0 || p < lo[0]) return -1;
  uint32_t a = 0, b = cnt;
  while (b - a > 1) {
    const uint32_t m = (a + b) >> 1;
    if (lo[m] <= p) a = m;
    else b = m;
  }
  return p < hi[a] ? (int)a : -1;
}


// every (bucket, record) entry of the valid records: counts (SCATTER false) or
// the bucket-sorted record list idx (SCATTER true, ctr = per-bucket cursors
// starting at the buckets' offsets)
template <bool SCATTER>
__device__ __forceinline__ void msm_bin(uint64_t n, const uint8_t* __restrict__ code, const uint8_t* __restrict__ inf,
                                        const MsmSegs& sg, const uint32_t* __restrict__ seed, uint64_t index_base,
                                        uint32_t* __restrict__ ctr, uint32_t* __restrict__ idx) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || code[i] != 0) return;
  int seg[2];
  if (!sg.pos) {
    seg[0] = 0;
    seg[1] = 1 + (int)sg.grp[i];
  } else {
    const uint32_t p = sg.pos[i];
    seg[0] = msm_find(sg.plo, sg.phi, sg.nparts, p);
    const int t = msm_find(sg.tlo, sg.thi, sg.nterms, p);
    seg[1] = t < 0 ? -1 : (int)sg.nparts + t;
  }
  if (seg[0] < 0 && seg[1] < 0) return;   // outside this check's ranges
  uint32_t k[4];
  rlc_scalar(seed, index_base + i, k);
  const uint8_t fl = inf[i];
#pragma unroll 1
  for (int set = 0; set < 2; set++) {
    if (seg[set] < 0 || (fl & (set ? INF_PK : INF_SIG))) continue;   // an identity term contributes nothing
    const uint32_t base = (uint32_t)seg[set] * MSM_SEG;
#pragma unroll 1
    for (uint32_t w = 0; w < MSM_WIN; w++) {
      const uint32_t d = msm_digit(k, w);
      if (!d) continue;
      if (SCATTER)
        idx[atomicAdd(&ctr[base + w * MSM_DIG + d], 1u)] = (uint32_t)i;
      else
        atomicAdd(&ctr[base + w * MSM_DIG + d], 1u);
    }
  }
}

__global__ CESS_LB void k_msm_count(uint64_t n, const uint8_t* __restrict__ code, const uint8_t* __restrict__ inf,
                                    MsmSegs sg, const uint32_t* __restrict__ seed, uint64_t index_base,
                                    uint32_t* __restrict__ counts) {
  msm_bin<false>(n, code, inf, sg, seed, index_base, counts, nullptr);
}
__global__ CESS_LB void k_msm_scatter(uint64_t n, const uint8_t* __restrict__ code, const uint8_t* __restrict__ inf,
                                      MsmSegs sg, const uint32_t* __restrict__ seed, uint64_t index_base,
                                      uint32_t* __restrict__ cursor, uint32_t* __restrict__ idx) {
  msm_bin<true>(n, code, inf, sg, seed, index_base, cursor, idx);
}

// pos[perm[j]] = j
__global__ void k_inv_perm(uint64_t n, const uint32_t* __restrict__ perm, uint32_t* __restrict__ pos) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j < n) pos[perm[j]] = (uint32_t)j;
}

// The batch's affine points record-major (24 words = 96 B per record), for
// the bucket gathers: a record's point is then 6 x 16-byte loads from two
// cache lines, where the SoA stage layout spreads it over 24 lines.
__global__ CESS_LB void k_msm_aos(uint64_t n, const uint32_t* __restrict__ X, uint4* __restrict__ Xa) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t w[24];
#pragma unroll
  for (int k = 0; k < 24; k++) w[k] = X[(uint64_t)k * n + i];
#pragma unroll
  for (int q = 0; q < 6; q++) Xa[6 * i + q] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
}

struct AffPt {
  uint4 v[6];
};
__device__ __forceinline__ AffPt ld_aff(const uint4* __restrict__ Xa, uint32_t i) {
  AffPt p;
#pragma unroll
  for (int q = 0; q < 6; q++) p.v[q] = Xa[6 * (uint64_t)i + q];
  return p;
}
__device__ __forceinline__ void aff_xy(const AffPt& p, fp& x, fp& y) {
#pragma unroll
  for (int q = 0; q < 3; q++) {
    x.v[4 * q] = p.v[q].x, x.v[4 * q + 1] = p.v[q].y, x.v[4 * q + 2] = p.v[q].z, x.v[4 * q + 3] = p.v[q].w;
    y.v[4 * q] = p.v[3 + q].x, y.v[4 * q + 1] = p.v[3 + q].y, y.v[4 * q + 2] = p.v[3 + q].z, y.v[4 * q + 3] = p.v[3 + q].w;
  }
}

// Work item j = one chunk of one bucket's entries (msm_chunk: >= 64 entries,
// <= 32 chunks per bucket; item_off = the buckets' first items, host-built):
// the chunk's points summed with mixed additions (record-major affine points,
// k_msm_aos; the parts' segments read the signatures Xs, the terms' the
// hashes Xh), the
// next entry's point loaded while the current one is added.
__global__ CESS_LB void k_msm_items(uint32_t n_items, uint32_t nb, uint32_t nparts, const uint32_t* __restrict__ item_off,
                                    const uint32_t* __restrict__ bstart, const uint32_t* __restrict__ bcnt,
                                    const uint32_t* __restrict__ idx, const uint4* __restrict__ Xs,
                                    const uint4* __restrict__ Xh, uint32_t* __restrict__ part, uint64_t pstride) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n_items) return;
  uint32_t lo = 0, hi = nb;   // the last bucket whose first item is <= j (non-empty)
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (item_off[mid] <= j) lo = mid;
    else hi = mid;
  }
  const uint32_t b = lo, cnt = bcnt[b], L = msm_chunk(cnt), t = j - item_off[b];
  const uint32_t s = bstart[b] + t * L, e = bstart[b] + min(cnt, (t + 1) * L);
  const uint4* X = b < nparts * MSM_SEG ? Xs : Xh;   // parts: signatures; terms: hashes
  g1p acc = proj_identity<fp>();
  AffPt nxt = ld_aff(X, idx[s]);
#pragma unroll 1
  for (uint32_t q = s; q < e; q++) {
    const AffPt cur = nxt;
    if (q + 1 < e) nxt = ld_aff(X, idx[q + 1]);
    fp x, y;
    aff_xy(cur, x, y);
    acc = proj_add_mixed(acc, x, y);
  }
  st_g1p(part, pstride, j, acc);
}

// bucket b = the sum of its items' partials (at most 32)
__global__ CESS_LB void k_msm_bucket_sum(uint32_t nb, const uint32_t* __restrict__ item_off,
                                         const uint32_t* __restrict__ part, uint64_t pstride,
                                         uint32_t* __restrict__ bsum) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nb) return;
  g1p acc = proj_identity<fp>();
#pragma unroll 1
  for (uint32_t j = item_off[b]; j < item_off[b + 1]; j++) acc = proj_add(acc, ld_g1p(part, pstride, j));
  st_g1p(bsum, nb, b, acc);
}

// lane t = (seg * 16 + w) * 16 + q: sum_{d in [16q, 16q + 16)} d B(seg, w, d)
// by a running sum over the 16 digits (B(., ., 0) is empty)
__global__ CESS_LB void k_msm_window(uint32_t nseg, const uint32_t* __restrict__ bsum, uint64_t nb,
                                     uint32_t* __restrict__ T) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x, nt = nseg * MSM_WIN * 16;
  if (t >= nt) return;
  const uint32_t sw = t >> 4, q = t & 15;
  g1p acc = proj_identity<fp>(), sum = proj_identity<fp>();
#pragma unroll 1
  for (int d = 16 * (int)q + 15; d >= 16 * (int)q; d--) {
    if (d) acc = proj_add(acc, ld_g1p(bsum, nb, sw * MSM_DIG + (uint32_t)d));
    sum = proj_add(sum, acc);
  }
  // sum = sum_d (d - 16q + 1) B_d, acc = sum_d B_d: add (16q - 1) acc
  const g1p corr = q ? proj_mul_u64(acc, 16 * q - 1) : proj_neg(acc);
  st_g1p(T, nt, t, proj_add(sum, corr));
}

// lane (seg, w): U(seg, w) = 2^(8w) sum_q T(seg, w, q)
__global__ CESS_LB void k_msm_wsum(uint32_t nseg, const uint32_t* __restrict__ T, uint32_t* __restrict__ U) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x, nu = nseg * MSM_WIN, nt = nu * 16;
  if (t >= nu) return;
  g1p acc = proj_identity<fp>();
#pragma unroll 1
  for (uint32_t q = 0; q < 16; q++) acc = proj_add(acc, ld_g1p(T, nt, t * 16 + q));
#pragma unroll 1
  for (uint32_t r = 0; r < 8 * (t % MSM_WIN); r++) acc = proj_dbl(acc);
  st_g1p(U, nu, t, acc);
}

// lane seg: S(seg) = sum_w U(seg, w); parts -> S[seg] (stride nparts), terms
// -> Qs[seg - nparts] (stride nterms)
__global__ CESS_LB void k_msm_finish(uint32_t nseg, uint32_t nparts, const uint32_t* __restrict__ U,
                                     uint32_t* __restrict__ S, uint32_t* __restrict__ Qs) {
  const uint32_t sg = blockIdx.x * blockDim.x + threadIdx.x, nu = nseg * MSM_WIN;
  if (sg >= nseg) return;
  g1p acc = proj_identity<fp>();
#pragma unroll 1
  for (uint32_t w = 0; w < MSM_WIN; w++) acc = proj_add(acc, ld_g1p(U, nu, sg * MSM_WIN + w));
  if (sg < nparts) st_g1p(S, nparts, sg, acc);
  else st_g1p(Qs, nseg - nparts, sg - nparts, acc);
}

// Segmented sums (batched bisection): segment q = perm positions
// [seg_off[q], seg_off[q] + seg_cnt[q]), B blocks per segment; block b =
// q * B + bx writes out[b] (SoA stride out_stride).  With perm = nullptr the
// positions index `in` directly (second pass over the partial sums).  1-D grid,
// so the segment count is not bound by gridDim.y.
__global__ __launch_bounds__(256, 1) void k_g1_sum_segs(uint32_t B, const uint64_t* __restrict__ seg_off,
                                                        const uint64_t* __restrict__ seg_cnt,
                                                        const uint32_t* __restrict__ perm, const uint32_t* __restrict__ in,
                                                        uint64_t in_stride, uint32_t* __restrict__ out,
                                                        uint64_t out_stride) {
  __shared__ uint32_t L[36][256];
  const uint32_t t = threadIdx.x, sg = blockIdx.x / B, bx = blockIdx.x % B;
  const uint64_t T = (uint64_t)B * blockDim.x, off = seg_off[sg], cnt = seg_cnt[sg];
  g1p acc = proj_identity<fp>();
#pragma unroll 1
  for (uint64_t j = (uint64_t)bx * blockDim.x + t; j < cnt; j += T) {
    const uint64_t idx = perm ? perm[off + j] : off + j;
    acc = proj_add(acc, ld_g1p(in, in_stride, (uint32_t)idx));
  }
#pragma unroll 1
  for (uint32_t s = 128; s >= 1; s >>= 1) {
    if (t >= s && t < 2 * s) {
      const fp* e = &acc.x;
#pragma unroll
      for (int w = 0; w < 3; w++)
#pragma unroll
        for (int l = 0; l < 12; l++) L[12 * w + l][t - s] = e[w].v[l];
    }
    __syncthreads();
    if (t < s) {
      g1p o;
      fp* e = &o.x;
#pragma unroll
      for (int w = 0; w < 3; w++)
#pragma unroll
        for (int l = 0; l < 12; l++) e[w].v[l] = L[12 * w + l][t];
      acc = proj_add(acc, o);
    }
    __syncthreads();
  }
  if (t == 0) st_g1p(out, out_stride, blockIdx.x, acc);
}

// Check records of a batched RLC check: term j (M terms, grouped by range)
// pairs (Q_j, pk_{group[j]}) and, for the first term of each range, also
// (S_{range[j]}, -G2).  pk_usable[g] = 0 for keys that are the identity
// (their pairing term is 1).  S: SoA stride NR (the number of ranges);
// Qs: stride M.  Output in k_miller's SoA input format
// (stride M); k_miller reads the key rows through cidx = group.
__global__ void k_rlc_pairs_list(uint32_t M, uint32_t NR, const uint32_t* __restrict__ range, const uint32_t* __restrict__ group,
                                 const uint32_t* __restrict__ S, const uint8_t* __restrict__ pk_usable,
                                 uint8_t* __restrict__ code, uint8_t* __restrict__ inf, uint32_t* __restrict__ sig_aff,
                                 uint32_t* __restrict__ h_aff, const uint32_t* __restrict__ Qs) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= M) return;
  const uint32_t r = range[j];
  uint8_t f = 0;
  g1a s = {fp_zero(), fp_one(), true};
  if (j == 0 || range[j - 1] != r) s = proj_to_affine(ld_g1p(S, NR, r));
  if (s.inf) f |= INF_SIG;
  g1a h = proj_to_affine(ld_g1p(Qs, M, j));
  if (h.inf || !pk_usable[group[j]]) f |= INF_PK;
  st_fp(sig_aff, M, j, s.x);
  st_fp(sig_aff + 12 * M, M, j, s.y);
  st_fp(h_aff, M, j, h.x);
  st_fp(h_aff + 12 * M, M, j, h.y);
  inf[j] = f;
  code[j] = 0;
}

// acc slot r (stride NR) = prod of the Miller values fin[tbeg[r] .. tbeg[r+1])
// (fin stride M).  One 64-lane block per range: lane t multiplies every 64th
// value into its own slot of `part` (stride NR * 64), then a tree over the
// block; a range without terms gets one.  So a range with many key groups costs
// ceil(cnt / 64) + 6 serial Fp12 products, not cnt.
__global__ __launch_bounds__(64) void k_fp12_prod_segs(uint32_t NR, const uint32_t* __restrict__ tbeg,
                                                        const uint4* __restrict__ fin, uint64_t M,
                                                        uint4* __restrict__ part, uint4* __restrict__ acc) {
  const uint32_t r = blockIdx.x, t = threadIdx.x;
  if (r >= NR) return;
  const uint64_t ps = (uint64_t)NR * 64;
  const uint32_t b = tbeg[r], e = tbeg[r + 1];
  GlobF12 mine{part, ps, r * 64 + t};
  if (b + t < e) {
    copy12(mine, GlobF12{const_cast<uint4*>(fin), M, b + t});
#pragma unroll 1
    for (uint32_t j = b + t + 64; j < e; j += 64) mul12(mine, GlobF12{const_cast<uint4*>(fin), M, j});
  } else {
    set_one12(mine);
  }
#pragma unroll 1
  for (uint32_t s = 32; s >= 1; s >>= 1) {
    __syncthreads();
    if (t < s) mul12(mine, GlobF12{part, ps, r * 64 + t + s});
  }
  __syncthreads();
  if (t == 0) copy12(GlobF12{acc, NR, r}, mine);
}

// code[0] = 0 iff prod_{j < m} gt_j == 1; gts: m canonical Gt values (576 B,
// 12 big-endian Fp in tower order, the cess_bls_gt_batch format)
__global__ void k_gt_prod(uint32_t m, const uint8_t* __restrict__ gts, uint4* __restrict__ tmp,
                          uint8_t* __restrict__ code) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  GlobF12 a{tmp, 1, 0}, b{tmp + 36, 1, 0};
#pragma unroll 1
  for (uint32_t j = 0; j < m; j++) {
    const GlobF12& d = j ? b : a;
#pragma unroll 1
    for (int k = 0; k < 6; k++) {
      uint32_t w[24];
      const uint8_t* src = gts + 576 * (uint64_t)j + 96 * k;
#pragma unroll 1
      for (int t = 0; t < 24; t++)
        w[t] = ((uint32_t)src[4 * t] << 24) | ((uint32_t)src[4 * t + 1] << 16) | ((uint32_t)src[4 * t + 2] << 8) |
               src[4 * t + 3];
      fp2 e = {to_mont(raw_from_be_words(w)), to_mont(raw_from_be_words(w + 12))};
      d.st(k, e);
    }
    if (j) mul12(a, b);
  }
  code[0] = is_one12(a) ? CODE_OK : CODE_PAIRING;
}

// ---- distinct-key RLC (host_rlc.cpp rlcd_*) ---------------------------------
// Every record keeps its own Miller value f_i = Miller(Q_i, pk_i) (one pair per
// record); a range's check multiplies its records' f_i with Miller(S_r, -G2),
// S_r = sum r_i sig_i over the range.

// k_miller input for the records of one chunk: h = affine(Q_i) (stride n, from
// k_rlc_scale), pair 0 off (INF_SIG), pair 1 off when Q_i or the key is the
// identity.  Records with a decode code are skipped by k_miller.
__global__ CESS_LB void k_rlcd_records(uint64_t m, const uint8_t* __restrict__ code, const uint8_t* __restrict__ inf_in,
                                       const uint32_t* __restrict__ Q, uint64_t qstride, uint32_t* __restrict__ h_aff,
                                       uint8_t* __restrict__ inf_out, uint64_t stride) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  uint8_t f = INF_SIG;
  g1a h = {fp_zero(), fp_one(), true};
  if (code[i] == 0) {
    h = proj_to_affine(ld_g1p(Q, qstride, i));
    if (h.inf || (inf_in[i] & INF_PK)) f |= INF_PK;
  } else {
    f |= INF_PK;
  }
  st_fp(h_aff, stride, i, h.x);
  st_fp(h_aff + 12 * stride, stride, i, h.y);
  inf_out[i] = f;
}

// k_miller input for the ranges' S terms: sig = affine(S_r), pair 1 off
__global__ void k_rlcd_s_records(uint32_t NR, const uint32_t* __restrict__ S, uint8_t* __restrict__ code,
                                 uint8_t* __restrict__ inf, uint32_t* __restrict__ sig_aff) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= NR) return;
  const g1a s = proj_to_affine(ld_g1p(S, NR, r));
  st_fp(sig_aff, NR, r, s.x);
  st_fp(sig_aff + 12 * NR, NR, r, s.y);
  inf[r] = INF_PK | (s.inf ? INF_SIG : 0);
  code[r] = 0;
}

// out[j] (stride nch) = product of fin[i] (stride fs) over i in [lo[j], hi[j])
// with code[i] == 0 (code == nullptr: every i); an empty product is one
__global__ __launch_bounds__(256) void k_fp12_prod_chunks(uint32_t nch, const uint64_t* __restrict__ lo,
                                                          const uint64_t* __restrict__ hi,
                                                          const uint8_t* __restrict__ code, const uint4* __restrict__ fin,
                                                          uint64_t fs, uint4* __restrict__ out) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= nch) return;
  GlobF12 mine{out, nch, j};
  bool first = true;
#pragma unroll 1
  for (uint64_t i = lo[j]; i < hi[j]; i++) {
    if (code && code[i] != 0) continue;
    const GlobF12 src{const_cast<uint4*>(fin), fs, (uint32_t)i};
    if (first) copy12(mine, src);
    else mul12(mine, src);
    first = false;
  }
  if (first) set_one12(mine);
}

// a[r] <- a[r] * b[r]  (both stride NR)
__global__ void k_fp12_mul_each(uint32_t NR, uint4* __restrict__ a, const uint4* __restrict__ b) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= NR) return;
  mul12(GlobF12{a, NR, r}, GlobF12{const_cast<uint4*>(b), NR, r});
}
