// RSA PKCS#1 v1.5 verify, moduli of up to 2048 bits (RSA_L2048 28-bit limbs); one
// translation unit per size class so the (long) fully expanded product scans
// compile in parallel.  Algorithm and reference: k_rsa.hpp.
#include "k_rsa.hpp"

CESS_RSA_KERNEL(k_rsa_verify_2048, RSA_L2048, 2)
