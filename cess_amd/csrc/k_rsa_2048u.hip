// RSA PKCS#1 v1.5 verify, moduli of up to 2048 bits, key-uniform waves: the
// records of a wave share their key (k_rsa_scatter's key-sorted, wave-padded
// lists), so the modulus is a scalar operand.  Algorithm and reference:
// k_rsa.hpp.
#include "k_rsa.hpp"

CESS_RSA_KERNEL_U(k_rsa_verify_2048u, RSA_L2048, 2)
