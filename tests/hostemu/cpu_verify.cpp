// CPU BASELINE ONLY (bench.py cpu_baseline leg, tests): the build's kernel
// algorithms (cess_amd/csrc/bls/*.hpp, value-based Miller loop and final
// exponentiation of pairing.hpp) compiled for the host with -DCESS_HOSTEMU and
// run on std::thread x `threads` host cores, one signature per call, the same
// per-record semantics as verify_bls_signature (utils/verify-bls-signatures/
// src/lib.rs:243-247): decode sig (code 2), decode key (code 4), pairing
// check (code 5).  It is "the build's CPU path", NOT the reference crate
// (bls12_381 0.7.1 is Rust and cannot be built in this image).
// Never linked into the product library.
#include <string.h>

#include <mutex>
#include <thread>
#include <vector>

#include "../../cess_amd/csrc/bls/h2c.hpp"
#include "../../cess_amd/csrc/bls/pairing.hpp"

using namespace bls;

namespace {
coeff3 g_neg_g2[N_COEFFS];
std::once_flag g_once;

void init_neg_g2() {
  fp2 gx = {fp_from(c::G2_GEN_X0), fp_from(c::G2_GEN_X1)};
  fp2 gy = neg(fp2{fp_from(c::G2_GEN_Y0), fp_from(c::G2_GEN_Y1)});
  g2_prepare(gx, gy, [](int i, const coeff3& k) { g_neg_g2[i] = k; });
}

void be_words(const uint8_t* b, int nwords, uint32_t* w) {
  for (int i = 0; i < nwords; i++)
    w[i] = ((uint32_t)b[4 * i] << 24) | ((uint32_t)b[4 * i + 1] << 16) | ((uint32_t)b[4 * i + 2] << 8) | b[4 * i + 3];
}

uint8_t verify_one(const uint8_t* sig, const uint8_t* msg, uint32_t mlen, const uint8_t* pk) {
  uint32_t ws[12], wp[24];
  be_words(sig, 12, ws);
  be_words(pk, 24, wp);
  g1a s;
  if (!g1_decompress(ws, s)) return 2;
  g2a q;
  if (!g2_decompress(wp, q)) return 4;
  g1a h = hash_to_g1(msg, mlen);
  coeff3 pkc[N_COEFFS];
  fp2 qx = q.inf ? fp2{fp_from(c::G2_GEN_X0), fp_from(c::G2_GEN_X1)} : q.x;
  fp2 qy = q.inf ? fp2{fp_from(c::G2_GEN_Y0), fp_from(c::G2_GEN_Y1)} : q.y;
  g2_prepare(qx, qy, [&](int i, const coeff3& k) { pkc[i] = k; });
  fp12 f = miller_loop2(s, false, h, q.inf, [&](int pair, int i) { return pair ? pkc[i] : g_neg_g2[i]; });
  return is_one(final_exponentiation(f)) ? 0 : 5;
}
}  // namespace

extern "C" {
// n fixed-size records (48-B sigs, 96-B keys, msg_len-byte messages, packed);
// codes_out[i] = 0..5 as cess_bls_verify_batch.  Returns 0.
int cpu_verify_batch(uint64_t n, const uint8_t* sigs, const uint8_t* msgs, uint32_t msg_len, const uint8_t* pks,
                     uint8_t* codes_out, int threads) {
  std::call_once(g_once, init_neg_g2);
  if (threads < 1) threads = 1;
  std::vector<std::thread> pool;
  for (int t = 0; t < threads; t++)
    pool.emplace_back([=] {
      for (uint64_t i = t; i < n; i += threads)
        codes_out[i] = verify_one(sigs + 48 * i, msgs + (uint64_t)msg_len * i, msg_len, pks + 96 * i);
    });
  for (auto& th : pool) th.join();
  return 0;
}
}
