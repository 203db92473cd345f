// RSA PKCS#1 v1.5 verify, moduli of up to 1024 bits (RSA_L1024 28-bit limbs); one
// translation unit per size class so the (long) fully expanded product scans
// compile in parallel.  Algorithm and reference: k_rsa.hpp.
#include "k_rsa.hpp"

CESS_RSA_KERNEL(k_rsa_verify_1024, RSA_L1024, 2)
