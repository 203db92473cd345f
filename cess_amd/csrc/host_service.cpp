// Node-side services of include/cess_bls.h around the verification pipeline
// (SURVEY §8(f) ranks 1-3):
//
//  * cess_bls_deserialize_batch: Signature::deserialize / PublicKey::deserialize
//    (reference utils/verify-bls-signatures/src/lib.rs:138-152, :68-82) on
//    their own -- the decode kernels only, not the six-kernel pairing pipeline
//    (a single deserialize costs the decode's latency, ~2-5 ms, not ~30 ms).
//  * cess_bls_cache_*: the bounded verdict cache the node host function reads
//    and the node batcher fills (utils/cess-gpu-verify-runtime).  Entries are
//    keyed by SHA-256 over the length-prefixed (sig, msg, key) bytes, so a
//    record can only ever hit its own verdict; at capacity the oldest entries
//    are evicted first.  Records without a cached verdict are verified in ONE
//    batch (cess_bls_verify_batch_var); when that is impossible (no context,
//    infrastructure failure) they are reported CESS_BLS_CODE_UNAVAILABLE and
//    nothing is cached, so the caller's own path (the runtime's unchanged wasm
//    verifier) decides -- the cache never invents a verdict.
#include <deque>
#include <unordered_map>

#include "host.hpp"

using namespace cess_host;

#define ENTRY(c)                          \
  if (!(c)) return CESS_BLS_E_INVALID_ARG; \
  CtxLock lock_(c);                        \
  if (!lock_.ok()) return CESS_BLS_E_BUSY

// ---------------------------------------------------------------------------
// deserialize batch
// ---------------------------------------------------------------------------
static int deserialize_one(cess_bls_ctx* c, int kind, size_t n, const uint8_t* data, const uint64_t* offs,
                           uint8_t* codes_out) {
  const size_t w = kind == CESS_BLS_KIND_SIG ? 48 : 96;
  HIPCHK(hipSetDevice(c->device));
  hipStream_t s = c->stream;
  int r = order_begin(c, s);
  if (r) return r;
  const uint32_t strict = (c->flags & CESS_BLS_F_STRICT_IDENTITY) ? 1u : 0u;
  std::vector<uint8_t> fixed, pre;
  for (size_t off = 0; off < n; off += c->qcap) {
    const uint64_t m = std::min<uint64_t>(c->qcap, n - off);
    fixed.assign(m * w, 0);
    pre.assign(m, 0);
    for (uint64_t j = 0; j < m; j++) {
      const uint64_t a = offs[off + j], b = offs[off + j + 1];
      if (b < a) return CESS_BLS_E_INVALID_ARG;
      if (b - a == w) memcpy(&fixed[j * w], data + a, w);
      else pre[j] = kind == CESS_BLS_KIND_SIG ? PRE_SIG_LEN_BAD : PRE_PK_LEN_BAD;
    }
    StageSlot& S = c->slot[0];
    r = c->in_sigs.ensure(m * w) | c->pre.ensure(m) | S.inf.ensure(c->qcap);
    if (kind == CESS_BLS_KIND_SIG) r |= S.sig_aff.ensure(c->qcap * CESS_W_G1 * 4);
    else r |= S.pk_aff.ensure(c->qcap * CESS_W_G2 * 4) | S.coeffs.ensure(c->qcap * (uint64_t)CESS_W_COEFFS * 4);
    if (r) return CESS_BLS_E_OOM;
    HIPCHK(hipMemcpyAsync(c->in_sigs.p, fixed.data(), m * w, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(c->pre.p, pre.data(), m, hipMemcpyHostToDevice, s));
    const unsigned g = grid_for(m);
    uint8_t* code = c->code.as<uint8_t>();
    uint8_t* inf = S.inf.as<uint8_t>();
    if (kind == CESS_BLS_KIND_SIG) {
      hipLaunchKernelGGL(k_decode_sig, dim3(g), dim3(kBlock), 0, s, m, c->in_sigs.as<uint8_t>(),
                         (const uint8_t*)c->pre.as<uint8_t>(), code, inf, S.sig_aff.as<uint32_t>(), c->qcap);
    } else {
      // k_decode_pk only touches records whose code is still 0 (the reference
      // precedence of a full verification); alone, every record starts at 0
      HIPCHK(hipMemsetAsync(code, 0, m, s));
      HIPCHK(hipMemsetAsync(inf, 0, m, s));
      hipLaunchKernelGGL(k_decode_pk, dim3(g), dim3(kBlock), 0, s, m, c->in_sigs.as<uint8_t>(),
                         (const uint8_t*)c->pre.as<uint8_t>(), code, inf, S.pk_aff.as<uint32_t>(), c->qcap, strict);
      // the subgroup check: psi(Q) == -[|x|]Q on the G2Prepared iteration's point
      hipLaunchKernelGGL(k_prepare, dim3(g), dim3(kBlock), 0, s, m, (const uint32_t*)S.pk_aff.as<uint32_t>(),
                         S.coeffs.as<uint4>(), c->qcap, code, (const uint8_t*)inf);
    }
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(codes_out + off, code, m, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));   // fixed / pre are reused by the next chunk
  }
  return order_end(c, s);
}

extern "C" int cess_bls_deserialize_batch(cess_bls_ctx* c, int kind, size_t n, const uint8_t* data,
                                          const uint64_t* offsets, uint8_t* codes_out) {
  ENTRY(c);
  if (kind != CESS_BLS_KIND_SIG && kind != CESS_BLS_KIND_PK) return CESS_BLS_E_INVALID_ARG;
  if (n && (!offsets || !codes_out || (!data && offsets[n] != offsets[0]))) return CESS_BLS_E_INVALID_ARG;
  if (n == 0) return CESS_BLS_OK;
  cess_bls_ctx* d = c->subs.empty() ? c : c->subs[0];
  return deserialize_one(d, kind, n, data, offsets, codes_out);
}

// ---------------------------------------------------------------------------
// SHA-256 (FIPS 180-4) for the cache keys (host)
// ---------------------------------------------------------------------------
namespace {

struct Sha256 {
  uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  uint8_t buf[64];
  size_t used = 0;
  uint64_t total = 0;

  static uint32_t rotr(uint32_t x, int r) { return (x >> r) | (x << (32 - r)); }

  void block(const uint8_t* p) {
    static const uint32_t K[64] = {
        0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
        0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
        0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
        0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
        0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
        0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
        0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
        0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
    uint32_t w[64];
    for (int i = 0; i < 16; i++)
      w[i] = ((uint32_t)p[4 * i] << 24) | ((uint32_t)p[4 * i + 1] << 16) | ((uint32_t)p[4 * i + 2] << 8) | p[4 * i + 3];
    for (int i = 16; i < 64; i++) {
      const uint32_t s0 = rotr(w[i - 15], 7) ^ rotr(w[i - 15], 18) ^ (w[i - 15] >> 3);
      const uint32_t s1 = rotr(w[i - 2], 17) ^ rotr(w[i - 2], 19) ^ (w[i - 2] >> 10);
      w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
    for (int i = 0; i < 64; i++) {
      const uint32_t t1 = hh + (rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25)) + ((e & f) ^ (~e & g)) + K[i] + w[i];
      const uint32_t t2 = (rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
      hh = g, g = f, f = e, e = d + t1, d = c, c = b, b = a, a = t1 + t2;
    }
    h[0] += a, h[1] += b, h[2] += c, h[3] += d, h[4] += e, h[5] += f, h[6] += g, h[7] += hh;
  }
  void update(const uint8_t* p, size_t n) {
    total += n;
    while (n) {
      const size_t k = std::min(n, 64 - used);
      memcpy(buf + used, p, k);
      used += k, p += k, n -= k;
      if (used == 64) {
        block(buf);
        used = 0;
      }
    }
  }
  void final(uint8_t out[32]) {
    const uint64_t bits = total * 8;
    const uint8_t one = 0x80, zero = 0;
    update(&one, 1);
    while (used != 56) update(&zero, 1);
    uint8_t len[8];
    for (int i = 0; i < 8; i++) len[i] = (uint8_t)(bits >> (56 - 8 * i));
    update(len, 8);
    for (int i = 0; i < 8; i++)
      for (int j = 0; j < 4; j++) out[4 * i + j] = (uint8_t)(h[i] >> (24 - 8 * j));
  }
};

struct Digest {
  uint8_t b[32];
  bool operator==(const Digest& o) const { return memcmp(b, o.b, 32) == 0; }
};
struct DigestHash {
  size_t operator()(const Digest& d) const {
    size_t v;
    memcpy(&v, d.b, sizeof(v));
    return v;
  }
};

// key of one record: SHA-256(u64le(|sig|) sig u64le(|msg|) msg u64le(|key|) key)
Digest record_digest(const uint8_t* sig, uint64_t sl, const uint8_t* msg, uint64_t ml, const uint8_t* key,
                     uint64_t kl) {
  Sha256 h;
  for (auto part : {std::make_pair(sig, sl), std::make_pair(msg, ml), std::make_pair(key, kl)}) {
    uint8_t len[8];
    for (int i = 0; i < 8; i++) len[i] = (uint8_t)(part.second >> (8 * i));
    h.update(len, 8);
    if (part.second) h.update(part.first, part.second);
  }
  Digest d;
  h.final(d.b);
  return d;
}

}  // namespace

extern "C" int cess_bls_sha256(const uint8_t* data, size_t len, uint8_t out[32]) {
  if ((!data && len) || !out) return CESS_BLS_E_INVALID_ARG;
  Sha256 h;
  if (len) h.update(data, len);
  h.final(out);
  return CESS_BLS_OK;
}

// ---------------------------------------------------------------------------
// verdict cache
// ---------------------------------------------------------------------------
struct cess_bls_cache {
  std::mutex mu;
  size_t capacity = 0;
  std::unordered_map<Digest, uint8_t, DigestHash> map;
  std::deque<Digest> order;   // insertion order, oldest first
  uint64_t evicted = 0;

  // insert or refresh; evicts the oldest entries beyond capacity
  uint64_t put(const Digest& d, uint8_t code) {
    auto it = map.find(d);
    if (it != map.end()) {
      it->second = code;
      return 0;
    }
    map.emplace(d, code);
    order.push_back(d);
    uint64_t ev = 0;
    while (map.size() > capacity) {
      map.erase(order.front());
      order.pop_front();
      ev++;
    }
    evicted += ev;
    return ev;
  }
};

extern "C" int cess_bls_cache_create(size_t capacity, cess_bls_cache** out) {
  if (!out || capacity == 0) return CESS_BLS_E_INVALID_ARG;
  *out = new cess_bls_cache();
  (*out)->capacity = capacity;
  return CESS_BLS_OK;
}

extern "C" void cess_bls_cache_destroy(cess_bls_cache* cache) { delete cache; }

extern "C" int cess_bls_cache_clear(cess_bls_cache* cache) {
  if (!cache) return CESS_BLS_E_INVALID_ARG;
  std::lock_guard<std::mutex> g(cache->mu);
  cache->map.clear();
  cache->order.clear();
  return CESS_BLS_OK;
}

extern "C" size_t cess_bls_cache_size(cess_bls_cache* cache) {
  if (!cache) return 0;
  std::lock_guard<std::mutex> g(cache->mu);
  return cache->map.size();
}

static bool offsets_ok(size_t n, const uint64_t* o) {
  for (size_t i = 0; i < n; i++)
    if (o[i + 1] < o[i]) return false;
  return true;
}
// a data buffer may be null only if its records are all empty
static bool data_ok(size_t n, const uint8_t* d, const uint64_t* o) { return d || o[n] == o[0]; }

extern "C" int cess_bls_cache_insert_var(cess_bls_cache* cache, size_t n, const uint8_t* sig_data,
                                         const uint64_t* sig_offsets, const uint8_t* pk_data,
                                         const uint64_t* pk_offsets, const uint8_t* msgs,
                                         const uint64_t* msg_offsets, const uint8_t* codes) {
  if (!cache) return CESS_BLS_E_INVALID_ARG;
  if (n == 0) return CESS_BLS_OK;
  if (!sig_offsets || !pk_offsets || !msg_offsets || !codes || !offsets_ok(n, sig_offsets) ||
      !offsets_ok(n, pk_offsets) || !offsets_ok(n, msg_offsets) || !data_ok(n, sig_data, sig_offsets) ||
      !data_ok(n, pk_data, pk_offsets) || !data_ok(n, msgs, msg_offsets))
    return CESS_BLS_E_INVALID_ARG;
  for (size_t i = 0; i < n; i++)
    if (codes[i] > CESS_BLS_CODE_PAIRING_FAIL) return CESS_BLS_E_INVALID_ARG;   // verdicts only
  std::vector<Digest> dg(n);
  for (size_t i = 0; i < n; i++)
    dg[i] = record_digest(sig_data + sig_offsets[i], sig_offsets[i + 1] - sig_offsets[i], msgs + msg_offsets[i],
                          msg_offsets[i + 1] - msg_offsets[i], pk_data + pk_offsets[i],
                          pk_offsets[i + 1] - pk_offsets[i]);
  std::lock_guard<std::mutex> g(cache->mu);
  for (size_t i = 0; i < n; i++) cache->put(dg[i], codes[i]);
  return CESS_BLS_OK;
}

extern "C" int cess_bls_cache_verify_var(cess_bls_cache* cache, cess_bls_ctx* ctx, size_t n, const uint8_t* sig_data,
                                         const uint64_t* sig_offsets, const uint8_t* pk_data,
                                         const uint64_t* pk_offsets, const uint8_t* msgs,
                                         const uint64_t* msg_offsets, uint8_t* codes_out, uint64_t* stats3) {
  if (!cache) return CESS_BLS_E_INVALID_ARG;
  if (stats3) stats3[0] = stats3[1] = stats3[2] = 0;
  if (n == 0) return CESS_BLS_OK;
  if (!sig_offsets || !pk_offsets || !msg_offsets || !codes_out || !offsets_ok(n, sig_offsets) ||
      !offsets_ok(n, pk_offsets) || !offsets_ok(n, msg_offsets) || !data_ok(n, sig_data, sig_offsets) ||
      !data_ok(n, pk_data, pk_offsets) || !data_ok(n, msgs, msg_offsets))
    return CESS_BLS_E_INVALID_ARG;
  std::vector<Digest> dg(n);
  for (size_t i = 0; i < n; i++)
    dg[i] = record_digest(sig_data + sig_offsets[i], sig_offsets[i + 1] - sig_offsets[i], msgs + msg_offsets[i],
                          msg_offsets[i + 1] - msg_offsets[i], pk_data + pk_offsets[i],
                          pk_offsets[i + 1] - pk_offsets[i]);
  // 1. hits; misses deduplicated (a record repeated in the batch is verified once)
  std::vector<size_t> miss;                    // first occurrence of each missing record
  std::vector<size_t> dup_of(n, SIZE_MAX);     // later occurrences -> index into miss
  uint64_t hits = 0;
  {
    std::lock_guard<std::mutex> g(cache->mu);
    std::unordered_map<Digest, size_t, DigestHash> first;
    for (size_t i = 0; i < n; i++) {
      auto it = cache->map.find(dg[i]);
      if (it != cache->map.end()) {
        codes_out[i] = it->second;
        hits++;
        continue;
      }
      auto f = first.find(dg[i]);
      if (f != first.end()) {
        dup_of[i] = f->second;
        continue;
      }
      first.emplace(dg[i], miss.size());
      dup_of[i] = miss.size();
      miss.push_back(i);
    }
  }
  if (stats3) stats3[0] = hits;
  if (miss.empty()) return CESS_BLS_OK;
  // 2. one variable-length batch for the misses
  const size_t m = miss.size();
  std::vector<uint8_t> sd, pd, md, mc(m, CESS_BLS_CODE_UNAVAILABLE);
  std::vector<uint64_t> so = {0}, po = {0}, mo = {0};
  for (size_t i : miss) {
    sd.insert(sd.end(), sig_data + sig_offsets[i], sig_data + sig_offsets[i + 1]);
    pd.insert(pd.end(), pk_data + pk_offsets[i], pk_data + pk_offsets[i + 1]);
    md.insert(md.end(), msgs + msg_offsets[i], msgs + msg_offsets[i + 1]);
    so.push_back(sd.size()), po.push_back(pd.size()), mo.push_back(md.size());
  }
  static const uint8_t zero = 0;
  int st = ctx ? cess_bls_verify_batch_var(ctx, m, sd.empty() ? &zero : sd.data(), so.data(),
                                           pd.empty() ? &zero : pd.data(), po.data(), md.empty() ? &zero : md.data(),
                                           mo.data(), mc.data(), nullptr)
               : CESS_BLS_E_NO_DEVICE;
  if (st != CESS_BLS_OK) std::fill(mc.begin(), mc.end(), CESS_BLS_CODE_UNAVAILABLE);
  for (size_t i = 0; i < n; i++)
    if (dup_of[i] != SIZE_MAX) codes_out[i] = mc[dup_of[i]];
  // 3. verdicts (never "unavailable") into the cache
  if (st == CESS_BLS_OK) {
    std::lock_guard<std::mutex> g(cache->mu);
    uint64_t ev = 0;
    for (size_t q = 0; q < m; q++) ev += cache->put(dg[miss[q]], mc[q]);
    if (stats3) stats3[1] = m, stats3[2] = ev;
  }
  return st;
}
