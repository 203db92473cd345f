// Host side of the RSA PKCS#1 v1.5 raw batch verifier:
// cp_enclave_verify::verify_rsa (reference primitives/enclave-verify/src/
// lib.rs:221-228) = RsaPublicKey::from_public_key_der(key).unwrap() then
// pk.verify(Pkcs1v15Sign::new_raw(), msg, sig) (rsa 0.8.2, not vendored).
//
// Per distinct key the host parses the DER (SubjectPublicKeyInfo, as
// from_public_key_der; or PKCS#1 RSAPublicKey, the 270-byte Podr2Key of
// primitives/common/src/lib.rs:54) and precomputes the Montgomery constants
// (n in 28-bit limbs, -n^-1 mod 2^28, R^2 mod n); every signature is checked
// on the GPU (k_rsa_classify + k_rsa_verify_{1024,2048}; few-key batches:
// k_rsa_count / _scan / _scatter + k_rsa_verify_2048u).
#include "host.hpp"
#include "rsa.hpp"

using namespace cess_host;

__global__ void k_rsa_classify(uint64_t, const uint32_t*, uint32_t, const RsaKeyDev*, const uint8_t*, const uint64_t*,
                               const uint64_t*, uint8_t*, uint32_t*, uint32_t*);
#define RSA_KERNEL_DECL(NAME)                                                                                        \
  __global__ void NAME(uint32_t, const uint32_t*, const uint32_t*, const uint32_t*, const RsaKeyDev*, const uint8_t*, \
                       const uint64_t*, const uint8_t*, const uint64_t*, uint32_t*, uint8_t*);
RSA_KERNEL_DECL(k_rsa_verify_1024)
RSA_KERNEL_DECL(k_rsa_verify_2048)
RSA_KERNEL_DECL(k_rsa_verify_2048u)
__global__ void k_rsa_verify_big(uint32_t, const uint32_t*, const uint32_t*, const uint32_t*, const RsaKeyDev*,
                                 const uint8_t*, const uint64_t*, const uint8_t*, const uint64_t*, uint8_t*);
__global__ void k_rsa_count(uint64_t, const uint32_t*, uint32_t, const RsaKeyDev*, const uint8_t*, const uint64_t*,
                            const uint64_t*, uint8_t*, uint32_t*);
__global__ void k_rsa_scan(uint32_t, const uint32_t*, uint32_t*, uint32_t*);
__global__ void k_rsa_scatter(uint64_t, const uint32_t*, uint32_t, const RsaKeyDev*, const uint8_t*, const uint64_t*,
                              const uint64_t*, const uint32_t*, uint32_t*, uint32_t*, uint64_t);
// key-uniform lists when the table has at most this many keys and the batch at
// least this many records per key (padding each (class, key) segment to a
// multiple of 64 then costs < 25 % idle lanes in the worst case)
constexpr uint32_t kRsaUniformMaxKeys = 4096;
constexpr uint64_t kRsaUniformMinPerKey = 256;

namespace {

constexpr uint32_t M28 = 0x0fffffffu;
const uint8_t kRsaOid[9] = {0x2a, 0x86, 0x48, 0x86, 0xf7, 0x0d, 0x01, 0x01, 0x01};   // 1.2.840.113549.1.1.1

// --- minimal DER (definite, minimal lengths) ---------------------------------
struct Tlv {
  uint8_t tag = 0;
  const uint8_t* v = nullptr;
  size_t len = 0, end = 0;
};

bool tlv(const uint8_t* b, size_t n, size_t pos, Tlv& t) {
  if (pos + 2 > n) return false;
  t.tag = b[pos];
  size_t ln = b[pos + 1];
  pos += 2;
  if (ln & 0x80) {
    const size_t nb = ln & 0x7f;
    if (nb == 0 || nb > 4 || pos + nb > n || b[pos] == 0) return false;
    ln = 0;
    for (size_t q = 0; q < nb; q++) ln = (ln << 8) | b[pos + q];
    if (ln < 0x80) return false;
    pos += nb;
  }
  if (pos + ln > n) return false;
  t.v = b + pos;
  t.len = ln;
  t.end = pos + ln;
  return true;
}

// non-negative minimal INTEGER -> big-endian magnitude without leading zeros
bool der_uint(const Tlv& t, std::vector<uint8_t>& out) {
  if (t.tag != 0x02 || t.len == 0 || (t.v[0] & 0x80)) return false;
  if (t.len > 1 && t.v[0] == 0 && !(t.v[1] & 0x80)) return false;
  size_t s = 0;
  while (s < t.len && t.v[s] == 0) s++;
  out.assign(t.v + s, t.v + t.len);
  return true;
}

bool parse_pkcs1(const uint8_t* b, size_t n, std::vector<uint8_t>& mod, uint64_t& e) {
  Tlv seq, tn, te;
  if (!tlv(b, n, 0, seq) || seq.tag != 0x30 || seq.end != n) return false;
  if (!tlv(seq.v, seq.len, 0, tn) || !tlv(seq.v, seq.len, tn.end, te) || te.end != seq.len) return false;
  std::vector<uint8_t> eb;
  if (!der_uint(tn, mod) || !der_uint(te, eb)) return false;
  if (eb.size() > 8) return false;
  e = 0;
  for (uint8_t v : eb) e = (e << 8) | v;
  // rsa 0.8 key checks (RsaPublicKey::new -> check_public): n at most 4096
  // bits, 2 <= e <= 2^33 - 1.  Keys the crate accepts but this verifier cannot
  // represent (even or tiny moduli) are reported by kernel_can_verify, not here.
  if (mod.empty() || mod.size() > 512) return false;
  if (e < 2 || e > (1ull << 33) - 1) return false;
  return true;
}

// Montgomery arithmetic needs an odd modulus > 2: other moduli that parse are
// CESS_RSA_E_UNSUPPORTED (the caller's CPU path decides), never BAD_KEY, so a
// GPU node cannot turn a key the rsa crate accepts into a rejection
bool kernel_can_verify(const std::vector<uint8_t>& mod) {
  return (mod.back() & 1) && !(mod.size() == 1 && mod[0] < 3);
}

// *unsup: the AlgorithmIdentifier carries parameters other than NULL (the
// crate's acceptance of those is unpinned here: reported as unsupported)
bool parse_spki(const uint8_t* b, size_t n, std::vector<uint8_t>& mod, uint64_t& e, bool* unsup) {
  Tlv seq, alg, bits, oid, nul;
  if (!tlv(b, n, 0, seq) || seq.tag != 0x30 || seq.end != n) return false;
  if (!tlv(seq.v, seq.len, 0, alg) || alg.tag != 0x30) return false;
  if (!tlv(seq.v, seq.len, alg.end, bits) || bits.tag != 0x03 || bits.end != seq.len) return false;
  if (!tlv(alg.v, alg.len, 0, oid) || oid.tag != 0x06 || oid.len != sizeof(kRsaOid) ||
      memcmp(oid.v, kRsaOid, sizeof(kRsaOid)) != 0)
    return false;
  if (oid.end != alg.len) {
    if (!tlv(alg.v, alg.len, oid.end, nul) || nul.end != alg.len) return false;
    if (nul.tag != 0x05 || nul.len != 0) *unsup = true;
  }
  if (bits.len < 1 || bits.v[0] != 0) return false;
  return parse_pkcs1(bits.v + 1, bits.len - 1, mod, e);
}

// limbs of the key's size class.  Every class must satisfy BOTH
//   28 L >= bits + 2  (R = 2^(28 L) >= 4n) and
//   28 L >= 8 k       (every bit of a k-byte signature has a limb, so the
//                      s < n check sees all of it: a 1033-bit key has 130-byte
//                      signatures, 1040 bits > 28 x 37, and s + 2^1036 would
//                      otherwise pass as s)
// The expanded 1024 / 2048-bit classes when they qualify, else the loop-form
// class (k_rsa_verify_big): the least multiple of RSA_BIG_ROWS with
// 28 L >= 8 k + 2, which implies both.
int size_class_limbs(size_t bits, size_t k_bytes) {
  auto fits = [&](int L) { return bits + 2 <= (size_t)28 * L && 8 * k_bytes <= (size_t)28 * L; };
  if (fits(RSA_L1024)) return RSA_L1024;
  if (fits(RSA_L2048)) return RSA_L2048;
  const int L0 = (int)((8 * k_bytes + 2 + 27) / 28);
  const int L = (L0 + RSA_BIG_ROWS - 1) / RSA_BIG_ROWS * RSA_BIG_ROWS;
  return L0 <= RSA_L4096 ? L : 0;
}

// big-endian bytes -> L 28-bit limbs (little-endian)
void to_limbs(const std::vector<uint8_t>& be, int L, uint32_t* out) {
  for (int q = 0; q < L; q++) out[q] = 0;
  const size_t nb = be.size();
  for (size_t i = 0; i < nb; i++) {   // byte i from the least significant end
    const uint32_t v = be[nb - 1 - i];
    const size_t bit = 8 * i, li = bit / 28, sh = bit % 28;
    if (li < (size_t)L) out[li] |= (v << sh) & M28;
    if (sh > 20 && li + 1 < (size_t)L) out[li + 1] |= v >> (28 - sh);
  }
}

// RsaKeyDev row of one parsed key (n odd, limbs = its size class)
void key_row(const std::vector<uint8_t>& mod, uint64_t e, int L, RsaKeyDev& k) {
  memset(&k, 0, sizeof(k));
  k.k_bytes = (uint32_t)mod.size();
  k.limbs = (uint32_t)L;
  k.e = e;
  to_limbs(mod, L, k.n28);
  // -n^-1 mod 2^28 (Newton: each step doubles the correct low bits)
  uint32_t inv = k.n28[0];
  for (int s = 0; s < 5; s++) inv *= 2u - k.n28[0] * inv;
  k.ninv = (0u - inv) & M28;
  // R^2 mod n, R = 2^(28 L): 2 * 28 L modular doublings of 1
  std::vector<uint32_t> x(L + 1, 0);
  x[0] = 1;
  for (int it = 0; it < 2 * 28 * L; it++) {
    uint32_t c = 0;
    for (int q = 0; q <= L; q++) {
      const uint32_t v = (x[q] << 1) | c;
      c = v >> 28;
      x[q] = v & M28;
    }
    // x < 2n: subtract n once if x >= n
    bool ge = true;
    for (int q = L; q >= 0; q--) {
      const uint32_t nq = q < L ? k.n28[q] : 0;
      if (x[q] != nq) {
        ge = x[q] > nq;
        break;
      }
    }
    if (ge) {
      int32_t br = 0;
      for (int q = 0; q <= L; q++) {
        const int32_t d = (int32_t)x[q] - (int32_t)(q < L ? k.n28[q] : 0) - br;
        br = d < 0;
        x[q] = (uint32_t)d & M28;
      }
    }
  }
  for (int q = 0; q < L; q++) k.r2_28[q] = x[q];
}

}  // namespace

// per-context RSA key tables (host_rsa.cpp): the caller's and a one-key table
// for the cess_rsa_verify drop-in
struct RsaTable {
  DevBuf keys, ok;
  uint32_t n = 0;
  bool big = false;   // a key of the loop-form class (2049-4096 bits)
};
struct RsaState {
  RsaTable user, single;
  DevBuf lists, counts, base, in_idx, in_sigs, in_soffs, in_msgs, in_moffs, out_codes;
};

static RsaState& rsa_state(cess_bls_ctx* c) {
  if (!c->rsa) c->rsa = new RsaState();
  return *c->rsa;
}
void cess_rsa_state_free(cess_bls_ctx* c) {
  delete c->rsa;
  c->rsa = nullptr;
}

static int load_table(cess_bls_ctx* c, RsaTable& T, size_t k, const uint8_t* ders, const uint64_t* offs, int format,
                      int* status_out) {
  std::vector<RsaKeyDev> rows(std::max<size_t>(k, 1));
  std::vector<uint8_t> ok(std::max<size_t>(k, 1), 0);
  bool big = false;
  for (size_t j = 0; j < k; j++) {
    std::vector<uint8_t> mod;
    uint64_t e = 0;
    const uint8_t* d = ders + offs[j];
    const size_t len = offs[j + 1] - offs[j];
    int st = CESS_BLS_OK;
    bool unsup = false;
    const bool parsed =
        format == CESS_RSA_KEY_PKCS1 ? parse_pkcs1(d, len, mod, e) : parse_spki(d, len, mod, e, &unsup);
    if (!parsed) st = CESS_BLS_E_BAD_KEY;
    else if (unsup || !kernel_can_verify(mod)) st = CESS_RSA_E_UNSUPPORTED;
    int L = 0;
    if (st == CESS_BLS_OK) {
      size_t bits = 8 * mod.size();
      for (uint8_t v = mod[0]; !(v & 0x80); v <<= 1) bits--;
      L = size_class_limbs(bits, mod.size());
      if (!L) st = CESS_RSA_E_UNSUPPORTED;
    }
    if (st == CESS_BLS_OK) {
      key_row(mod, e, L, rows[j]);
      ok[j] = 1;
      big = big || L > RSA_L2048;
    } else {
      memset(&rows[j], 0, sizeof(RsaKeyDev));
    }
    if (status_out) status_out[j] = st;
  }
  HIPCHK(hipSetDevice(c->device));
  if (T.keys.ensure(rows.size() * sizeof(RsaKeyDev)) | T.ok.ensure(ok.size())) return CESS_BLS_E_OOM;
  HIPCHK(hipMemcpy(T.keys.p, rows.data(), rows.size() * sizeof(RsaKeyDev), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(T.ok.p, ok.data(), ok.size(), hipMemcpyHostToDevice));
  T.n = (uint32_t)k;
  T.big = big;
  return CESS_BLS_OK;
}

// device-resident records against table T, enqueued on s
static int rsa_run(cess_bls_ctx* c, RsaTable& T, hipStream_t s, uint64_t n, const uint32_t* d_idx,
                   const uint8_t* d_sigs, const uint64_t* d_soffs, const uint8_t* d_msgs, const uint64_t* d_moffs,
                   uint8_t* d_codes) {
  if (n == 0) return CESS_BLS_OK;
  if (n >= (1ull << 31)) return CESS_BLS_E_INVALID_ARG;
  RsaState& S = rsa_state(c);
  if (T.keys.ensure(sizeof(RsaKeyDev)) | T.ok.ensure(1)) return CESS_BLS_E_OOM;
  const RsaKeyDev* K = T.keys.as<RsaKeyDev>();
  // Few keys with many records each (the TEE-key workload): key-sorted,
  // wave-padded lists, so each wave of the 2048-bit kernel has one key and its
  // modulus is a scalar operand (k_rsa_2048u).  Otherwise unsorted lists.
  if (!T.big && T.n > 0 && T.n <= kRsaUniformMaxKeys && n >= kRsaUniformMinPerKey * (uint64_t)T.n) {
    const uint64_t nk = T.n, cap = n + 64 * nk;   // each (class, key) segment pads < 64 entries
    if (S.lists.ensure(2 * cap * 4) | S.counts.ensure((6 * nk + 2) * 4) | S.base.ensure(cap * RSA_L2048 * 4))
      return CESS_BLS_E_OOM;
    uint32_t* cnt = S.counts.as<uint32_t>();
    uint32_t *cur = cnt + 2 * nk, *segbase = cnt + 4 * nk, *totals = cnt + 6 * nk;
    HIPCHK(hipMemsetAsync(cnt, 0, 4 * nk * 4, s));
    HIPCHK(hipMemsetAsync(S.lists.p, 0xff, 2 * cap * 4, s));   // RSA_PAD
    hipEvent_t a;
    int r = prof_begin(c, s, ST_RSA_CLASSIFY, &a);
    if (r) return r;
    hipLaunchKernelGGL(k_rsa_count, dim3(grid_for(n)), dim3(kBlock), 0, s, n, d_idx, T.n, K,
                       (const uint8_t*)T.ok.as<uint8_t>(), d_soffs, d_moffs, d_codes, cnt);
    hipLaunchKernelGGL(k_rsa_scan, dim3(1), dim3(64), 0, s, T.n, (const uint32_t*)cnt, segbase, totals);
    hipLaunchKernelGGL(k_rsa_scatter, dim3(grid_for(n)), dim3(kBlock), 0, s, n, d_idx, T.n, K,
                       (const uint8_t*)T.ok.as<uint8_t>(), d_soffs, d_moffs, (const uint32_t*)segbase, cur,
                       S.lists.as<uint32_t>(), cap);
    r = prof_end(c, s, ST_RSA_CLASSIFY, a);
    if (r) return r;
    const uint32_t* L = S.lists.as<uint32_t>();
    uint32_t* B = S.base.as<uint32_t>();
    r = prof_begin(c, s, ST_RSA_VERIFY, &a);
    if (r) return r;
    hipLaunchKernelGGL(k_rsa_verify_2048u, dim3(grid_for(cap)), dim3(kBlock), 0, s, (uint32_t)cap,
                       (const uint32_t*)(totals + 1), L + cap, d_idx, K, d_sigs, d_soffs, d_msgs, d_moffs, B, d_codes);
    hipLaunchKernelGGL(k_rsa_verify_1024, dim3(grid_for(cap)), dim3(kBlock), 0, s, (uint32_t)cap,
                       (const uint32_t*)totals, L, d_idx, K, d_sigs, d_soffs, d_msgs, d_moffs, B, d_codes);
    r = prof_end(c, s, ST_RSA_VERIFY, a);
    if (r) return r;
    HIPCHK(hipGetLastError());
    return CESS_BLS_OK;
  }
  if (S.lists.ensure(3 * n * 4) | S.counts.ensure(16) | S.base.ensure(n * RSA_L2048 * 4)) return CESS_BLS_E_OOM;
  HIPCHK(hipMemsetAsync(S.counts.p, 0, 16, s));
  // per-launch HIP events on s (CESS_BLS_F_PROFILE): bench.py's roofline
  // takes the verification kernel's duration from them
  hipEvent_t a;
  int r = prof_begin(c, s, ST_RSA_CLASSIFY, &a);
  if (r) return r;
  hipLaunchKernelGGL(k_rsa_classify, dim3(grid_for(n)), dim3(kBlock), 0, s, n, d_idx, T.n,
                     (const RsaKeyDev*)T.keys.as<RsaKeyDev>(), (const uint8_t*)T.ok.as<uint8_t>(), d_soffs, d_moffs,
                     d_codes, S.lists.as<uint32_t>(), S.counts.as<uint32_t>());
  r = prof_end(c, s, ST_RSA_CLASSIFY, a);
  if (r) return r;
  const uint32_t* cnt = S.counts.as<uint32_t>();
  const uint32_t* L = S.lists.as<uint32_t>();
  uint32_t* B = S.base.as<uint32_t>();
  // every class kernel covers n lanes; lanes past the class's count exit
  r = prof_begin(c, s, ST_RSA_VERIFY, &a);
  if (r) return r;
  hipLaunchKernelGGL(k_rsa_verify_2048, dim3(grid_for(n)), dim3(kBlock), 0, s, (uint32_t)n, cnt + 1, L + n, d_idx, K,
                     d_sigs, d_soffs, d_msgs, d_moffs, B, d_codes);
  hipLaunchKernelGGL(k_rsa_verify_1024, dim3(grid_for(n)), dim3(kBlock), 0, s, (uint32_t)n, cnt, L, d_idx, K, d_sigs,
                     d_soffs, d_msgs, d_moffs, B, d_codes);
  if (T.big)   // 2049-4096-bit moduli (list 2)
    hipLaunchKernelGGL(k_rsa_verify_big, dim3(grid_for(n)), dim3(kBlock), 0, s, (uint32_t)n, cnt + 2, L + 2 * n, d_idx,
                       K, d_sigs, d_soffs, d_msgs, d_moffs, d_codes);
  r = prof_end(c, s, ST_RSA_VERIFY, a);
  if (r) return r;
  HIPCHK(hipGetLastError());
  return CESS_BLS_OK;
}

static int rsa_host(cess_bls_ctx* c, RsaTable& T, size_t n, const uint32_t* key_idx, const uint8_t* sigs,
                    const uint64_t* soffs, const uint8_t* msgs, const uint64_t* moffs, uint8_t* codes_out,
                    uint64_t* bitmap_out) {
  if (n == 0) return CESS_BLS_OK;
  if (!key_idx || !soffs || !moffs) return CESS_BLS_E_INVALID_ARG;
  RsaState& S = rsa_state(c);
  HIPCHK(hipSetDevice(c->device));
  hipStream_t s = c->stream;
  int r = order_begin(c, s);
  if (r) return r;
  const uint64_t sb = soffs[n] - soffs[0], mb = moffs[n] - moffs[0];
  std::vector<uint64_t> so(n + 1), mo(n + 1);
  for (size_t i = 0; i <= n; i++) {
    if (i && (soffs[i] < soffs[i - 1] || moffs[i] < moffs[i - 1])) return CESS_BLS_E_INVALID_ARG;
    so[i] = soffs[i] - soffs[0];
    mo[i] = moffs[i] - moffs[0];
  }
  if (S.in_idx.ensure(n * 4) | S.in_sigs.ensure(std::max<uint64_t>(sb, 1)) | S.in_soffs.ensure((n + 1) * 8) |
      S.in_msgs.ensure(std::max<uint64_t>(mb, 1)) | S.in_moffs.ensure((n + 1) * 8) | S.out_codes.ensure(n))
    return CESS_BLS_E_OOM;
  HIPCHK(hipMemcpyAsync(S.in_idx.p, key_idx, n * 4, hipMemcpyHostToDevice, s));
  if (sb) HIPCHK(hipMemcpyAsync(S.in_sigs.p, sigs + soffs[0], sb, hipMemcpyHostToDevice, s));
  if (mb) HIPCHK(hipMemcpyAsync(S.in_msgs.p, msgs + moffs[0], mb, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(S.in_soffs.p, so.data(), (n + 1) * 8, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(S.in_moffs.p, mo.data(), (n + 1) * 8, hipMemcpyHostToDevice, s));
  r = rsa_run(c, T, s, n, S.in_idx.as<uint32_t>(), S.in_sigs.as<uint8_t>(), S.in_soffs.as<uint64_t>(),
              S.in_msgs.as<uint8_t>(), S.in_moffs.as<uint64_t>(), S.out_codes.as<uint8_t>());
  if (r) return r;
  r = collect_profile(c, s);
  if (r) return r;
  std::vector<uint8_t> codes(n);
  HIPCHK(hipMemcpyAsync(codes.data(), S.out_codes.p, n, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  if (codes_out) memcpy(codes_out, codes.data(), n);
  if (bitmap_out) bitmap_from_codes(codes.data(), n, bitmap_out);
  return order_end(c, s);
}

#define ENTRY(c)                          \
  if (!(c)) return CESS_BLS_E_INVALID_ARG; \
  CtxLock lock_(c);                        \
  if (!lock_.ok()) return CESS_BLS_E_BUSY

extern "C" int cess_rsa_parse_key(const uint8_t* der, size_t len, int format, uint8_t* n_out, size_t n_cap,
                                  size_t* n_len, uint64_t* e_out) {
  if ((!der && len) || !n_len || !e_out) return CESS_BLS_E_INVALID_ARG;
  std::vector<uint8_t> mod;
  uint64_t e = 0;
  bool unsup = false;   // not reported here: parse_key answers "does the crate parse it" (cess_rsa.h)
  const bool ok = format == CESS_RSA_KEY_PKCS1 ? parse_pkcs1(der, len, mod, e) : parse_spki(der, len, mod, e, &unsup);
  if (!ok) return CESS_BLS_E_BAD_KEY;
  *n_len = mod.size();
  *e_out = e;
  if (n_out) {
    if (n_cap < mod.size()) return CESS_BLS_E_INVALID_ARG;
    memcpy(n_out, mod.data(), mod.size());
  }
  return CESS_BLS_OK;
}

extern "C" int cess_rsa_keys_load(cess_bls_ctx* c, size_t k, const uint8_t* ders, const uint64_t* der_offsets,
                                  int format, int* key_status_out) {
  ENTRY(c);
  if ((k && (!ders || !der_offsets)) || k > 0xffffffffull) return CESS_BLS_E_INVALID_ARG;
  if (format != CESS_RSA_KEY_SPKI && format != CESS_RSA_KEY_PKCS1) return CESS_BLS_E_INVALID_ARG;
  if (c->subs.empty()) return load_table(c, rsa_state(c).user, k, ders, der_offsets, format, key_status_out);
  for (size_t d = 0; d < c->subs.size(); d++) {
    int r = load_table(c->subs[d], rsa_state(c->subs[d]).user, k, ders, der_offsets, format,
                       d == 0 ? key_status_out : nullptr);
    if (r) return r;
  }
  return CESS_BLS_OK;
}

int cess_multi_rsa(cess_bls_ctx* c, size_t n, const uint32_t* key_idx, const uint8_t* sigs, const uint64_t* soffs,
                   const uint8_t* msgs, const uint64_t* moffs, uint8_t* codes_out, uint64_t* bitmap_out);

int cess_rsa_one(cess_bls_ctx* s, size_t n, const uint32_t* key_idx, const uint8_t* sigs, const uint64_t* soffs,
                 const uint8_t* msgs, const uint64_t* moffs, uint8_t* codes_out, uint64_t* bitmap_out) {
  return rsa_host(s, rsa_state(s).user, n, key_idx, sigs, soffs, msgs, moffs, codes_out, bitmap_out);
}

extern "C" int cess_rsa_verify_batch(cess_bls_ctx* c, size_t n, const uint32_t* key_idx, const uint8_t* sigs,
                                     const uint64_t* sig_offsets, const uint8_t* msgs, const uint64_t* msg_offsets,
                                     uint8_t* codes_out, uint64_t* bitmap_out) {
  ENTRY(c);
  if (!c->subs.empty())
    return cess_multi_rsa(c, n, key_idx, sigs, sig_offsets, msgs, msg_offsets, codes_out, bitmap_out);
  return rsa_host(c, rsa_state(c).user, n, key_idx, sigs, sig_offsets, msgs, msg_offsets, codes_out, bitmap_out);
}

extern "C" int cess_rsa_verify_batch_device(cess_bls_ctx* c, size_t n, const uint32_t* d_key_idx, const uint8_t* d_sigs,
                                            const uint64_t* d_sig_offsets, const uint8_t* d_msgs,
                                            const uint64_t* d_msg_offsets, uint8_t* d_codes, void* stream) {
  ENTRY(c);
  if (!c->subs.empty() || (n && (!d_key_idx || !d_sig_offsets || !d_msg_offsets || !d_codes)))
    return CESS_BLS_E_INVALID_ARG;
  HIPCHK(hipSetDevice(c->device));
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  int r = order_begin(c, s);
  if (r) return r;
  r = rsa_run(c, rsa_state(c).user, s, n, d_key_idx, d_sigs, d_sig_offsets, d_msgs, d_msg_offsets, d_codes);
  if (r) return r;
  r = collect_profile(c, s);   // no-op without CESS_BLS_F_PROFILE
  if (r) return r;
  return order_end(c, s);
}

extern "C" int cess_rsa_verify(cess_bls_ctx* c, const uint8_t* key_der, size_t key_len, const uint8_t* msg,
                               size_t msg_len, const uint8_t* sig, size_t sig_len, int* ok_out) {
  ENTRY(c);
  if (!ok_out || (!key_der && key_len) || (!msg && msg_len) || (!sig && sig_len)) return CESS_BLS_E_INVALID_ARG;
  *ok_out = 0;
  cess_bls_ctx* d = c->subs.empty() ? c : c->subs[0];
  static const uint8_t zero = 0;
  const uint64_t ko[2] = {0, key_len};
  int st = CESS_BLS_OK;
  RsaTable& T = rsa_state(d).single;
  int r = load_table(d, T, 1, key_der ? key_der : &zero, ko, CESS_RSA_KEY_SPKI, &st);
  if (r) return r;
  if (st) return st;   // from_public_key_der(key).unwrap() would panic
  const uint32_t idx = 0;
  const uint64_t so[2] = {0, sig_len}, mo[2] = {0, msg_len};
  uint8_t code = 0xff;
  r = rsa_host(d, T, 1, &idx, sig ? sig : &zero, so, msg ? msg : &zero, mo, &code, nullptr);
  if (r) return r;
  *ok_out = code == RSA_OK;
  return CESS_BLS_OK;
}
