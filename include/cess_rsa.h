/*
 * cess_rsa.h -- C ABI of the MI355X batch RSA PKCS#1 v1.5 (raw) verifier
 * (SURVEY §8(f) rank 4), in the same library and context as cess_bls.h.
 *
 * Replaces cp_enclave_verify::verify_rsa (reference
 * primitives/enclave-verify/src/lib.rs:221-228):
 *     let pk = rsa::RsaPublicKey::from_public_key_der(key).unwrap();
 *     pk.verify(Pkcs1v15Sign::new_raw(), msg, sig).is_ok()
 * (rsa 0.8.2, Cargo.lock:6538-6541: RFC 8017 RSASSA-PKCS1-v1_5-VERIFY with no
 * DigestInfo prefix: EM = 0x00 0x01 0xff..0xff 0x00 || msg).
 *
 * Per-signature codes: 0 OK, 1 SIG_LEN (len != k), 2 SIG_RANGE (s >= n),
 * 3 MSG_LEN (k < len(msg) + 11), 4 MISMATCH, 5 KEY (no such key / the key did
 * not load).  Codes 1..5 are the reference's `false`.  Every modulus size
 * the crate accepts (up to 4096 bits) is verified on the GPU: 1024/2048-bit
 * size classes expanded at compile time (Podr2Key is a 2048-bit key) and a
 * loop-form kernel for 2049..4096 bits.  Keys the reference accepts but the
 * GPU cannot verify -- even moduli, n < 3, SPKI AlgorithmIdentifier
 * parameters other than NULL -- report CESS_RSA_E_UNSUPPORTED, never
 * CESS_BLS_E_BAD_KEY: the verdict path for them is the caller's (the node
 * hook answers "unavailable" and the runtime's unchanged
 * cp_enclave_verify::verify_rsa decides), so a GPU node never
 * turns a key the rsa crate accepts into a rejection.  BAD_KEY means the
 * crate's from_public_key_der fails too (malformed DER, > 4096 bits, e out of
 * [2, 2^33 - 1]).  Return values are infrastructure status as in cess_bls.h.
 */
#ifndef CESS_RSA_H
#define CESS_RSA_H

#include "cess_bls.h"

#ifdef __cplusplus
extern "C" {
#endif

#define CESS_RSA_E_UNSUPPORTED (-10) /* the key parses (the reference accepts it) but the GPU cannot verify it */

enum cess_rsa_code {
  CESS_RSA_OK = 0,
  CESS_RSA_SIG_LEN = 1,
  CESS_RSA_SIG_RANGE = 2,
  CESS_RSA_MSG_LEN = 3,
  CESS_RSA_MISMATCH = 4,
  CESS_RSA_KEY = 5
};

#define CESS_RSA_KEY_SPKI 0  /* SubjectPublicKeyInfo DER: what RsaPublicKey::from_public_key_der parses */
#define CESS_RSA_KEY_PKCS1 1 /* RSAPublicKey DER: Podr2Key = [u8; 270] (primitives/common/src/lib.rs:54) */

/* Host-side DER parse (the key checks of rsa 0.8: n <= 4096 bits,
 * 2 <= e <= 2^33 - 1).  n_out (may be NULL) receives the big-endian modulus
 * (*n_len bytes).  CESS_BLS_E_BAD_KEY where from_public_key_der fails.
 * This reports ONLY whether the reference crate parses the key: a key it
 * parses but the GPU kernels cannot verify (even or tiny modulus, SPKI
 * AlgorithmIdentifier parameters other than NULL) returns CESS_BLS_OK here and
 * CESS_RSA_E_UNSUPPORTED from cess_rsa_keys_load / cess_rsa_verify. */
int cess_rsa_parse_key(const uint8_t* der, size_t len, int format, uint8_t* n_out, size_t n_cap, size_t* n_len,
                       uint64_t* e_out);

/* Distinct-key table: k DER keys (key j = ders[der_offsets[j] .. [j+1]));
 * per key status (0, CESS_BLS_E_BAD_KEY, CESS_RSA_E_UNSUPPORTED) in
 * key_status_out (may be NULL).  Montgomery constants are precomputed once
 * per key.  Replaces the context's previous RSA table. */
int cess_rsa_keys_load(cess_bls_ctx* ctx, size_t k, const uint8_t* ders, const uint64_t* der_offsets, int format,
                       int* key_status_out);

/* verify_rsa over a batch: record i = (key key_idx[i], msg i, sig i), byte
 * ranges by offsets (n + 1 entries each).  codes_out (n) / bitmap_out
 * (ceil(n/64) words, bit = code 0) may be NULL.  Host buffers. */
int cess_rsa_verify_batch(cess_bls_ctx* ctx, size_t n, const uint32_t* key_idx, const uint8_t* sigs,
                          const uint64_t* sig_offsets, const uint8_t* msgs, const uint64_t* msg_offsets,
                          uint8_t* codes_out, uint64_t* bitmap_out);

/* Device-resident form (every pointer in HBM; offsets relative to d_sigs /
 * d_msgs); enqueued on `stream` (NULL: the context's), not synchronised. */
int cess_rsa_verify_batch_device(cess_bls_ctx* ctx, size_t n, const uint32_t* d_key_idx, const uint8_t* d_sigs,
                                 const uint64_t* d_sig_offsets, const uint8_t* d_msgs,
                                 const uint64_t* d_msg_offsets, uint8_t* d_codes, void* stream);

/* cp_enclave_verify::verify_rsa(key, msg, sig) drop-in: SPKI DER key;
 * CESS_BLS_E_BAD_KEY where from_public_key_der(key).unwrap() panics
 * (CESS_RSA_E_UNSUPPORTED for keys the GPU cannot verify, see above); else
 * *ok_out = the verdict. */
int cess_rsa_verify(cess_bls_ctx* ctx, const uint8_t* key_der, size_t key_len, const uint8_t* msg, size_t msg_len,
                    const uint8_t* sig, size_t sig_len, int* ok_out);

#ifdef __cplusplus
}
#endif
#endif /* CESS_RSA_H */
