// Shared definitions of the RSA PKCS#1 v1.5 verifier (k_rsa.hip, host_rsa.cpp).
#pragma once
#include <stdint.h>

// 28-bit limbs per size class: R = 2^(28 L) >= 4n for moduli of up to
// 1024 / 2048 bits (28 L >= bits + 2), expanded at compile time
// (k_rsa_verify_1024 / _2048 / _2048u).  Moduli of 2049-4096 bits (the rest of
// what rsa 0.8's from_public_key_der accepts) take the loop-form kernel
// k_rsa_verify_big with L = ceil((8 k + 2) / 28) limbs (k = byte length of n)
// rounded up to a multiple of RSA_BIG_ROWS (its Montgomery product runs that
// many rows per pass), chosen per key at run time (a fully expanded 3072-bit
// class, L = 110, took 28 minutes to compile).
#define RSA_L1024 37
#define RSA_L2048 74
#define RSA_L4096 147
#ifndef RSA_BIG_ROWS
#define RSA_BIG_ROWS 8
#endif
#define RSA_LMAX (((RSA_L4096 + RSA_BIG_ROWS - 1) / RSA_BIG_ROWS) * RSA_BIG_ROWS)

// an inactive entry of a wave-padded record list (k_rsa_scatter)
#define RSA_PAD 0xffffffffu

// verdict codes (oracle/rsa_oracle.py)
enum : uint8_t { RSA_OK = 0, RSA_SIG_LEN = 1, RSA_SIG_RANGE = 2, RSA_MSG_LEN = 3, RSA_MISMATCH = 4, RSA_KEY = 5 };

// one row of the device key table
struct RsaKeyDev {
  uint32_t k_bytes;       // byte length of n
  uint32_t ninv;          // -n^-1 mod 2^28
  uint32_t limbs;         // size class L
  uint32_t pad;
  uint64_t e;             // public exponent (2 <= e < 2^33)
  uint32_t n28[RSA_LMAX];     // n, 28-bit limbs, little-endian
  uint32_t r2_28[RSA_LMAX];   // R^2 mod n, R = 2^(28 L)
};
