// Host build of the loop-form RSA class's Montgomery product
// (cess_amd/csrc/rsa_mont.hpp) for tests/test_rsa.py.
#include "../../cess_amd/csrc/rsa_mont.hpp"

extern "C" void emu_rsa_mont(const uint32_t* a, const uint32_t* b, const uint32_t* n, uint32_t ninv, int L,
                             uint32_t* out) {
  rsa_big::mont_rt(a, b, n, ninv, L, out);
}
