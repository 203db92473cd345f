// Shared definitions of the RSA PKCS#1 v1.5 verifier (k_rsa.hip, host_rsa.cpp).
#pragma once
#include <stdint.h>

// 28-bit limbs per size class: R = 2^(28 L) >= 4n for moduli of up to
// 1024 / 2048 bits (28 L >= bits + 2).  (A 3072-bit class, L = 110, was built
// and took 28 minutes to compile as a fully expanded product scan; Podr2Key is
// 2048-bit, so larger keys report CESS_RSA_E_UNSUPPORTED.)
#define RSA_L1024 37
#define RSA_L2048 74
#define RSA_LMAX RSA_L2048

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
