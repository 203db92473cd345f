// Iterations of 30 divsteps until g == 0 for the 381-bit BLS12-381 p: the original
// variant (delta from 1) against the half-delta one (from 1/2), random inputs.
// Build: gcc -O2 tools/divsteps_sim.c -o /tmp/divsteps_sim && /tmp/divsteps_sim 200000
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include <stdlib.h>
typedef unsigned __int128 u128;
#define NW 7   // 64-bit words, signed two's complement 448 bits
typedef struct { int64_t w[NW]; } big;  // little-endian words, w[NW-1] signed
static void add(big* a, const big* b) { u128 c = 0; for (int i = 0; i < NW; i++) { c += (u128)(uint64_t)a->w[i] + (uint64_t)b->w[i]; a->w[i] = (int64_t)(uint64_t)c; c >>= 64; } }
static void sub(big* a, const big* b) { big nb; u128 c = 1; for (int i = 0; i < NW; i++) { c += (u128)(uint64_t)~b->w[i]; nb.w[i] = (int64_t)(uint64_t)c; c >>= 64; } add(a, &nb); }
static void shr1(big* a) { for (int i = 0; i < NW - 1; i++) a->w[i] = (int64_t)(((uint64_t)a->w[i] >> 1) | ((uint64_t)a->w[i + 1] << 63)); a->w[NW - 1] >>= 1; }
static int iszero(const big* a) { for (int i = 0; i < NW; i++) if (a->w[i]) return 0; return 1; }
static uint64_t rng = 88172645463325252ull; static uint64_t xr(void) { rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17; return rng; }
int main(int argc, char** argv) {
  const uint64_t P[6] = {0xb9feffffffffaaabull, 0x1eabfffeb153ffffull, 0x6730d2a0f6b0f624ull, 0x64774b84f38512bfull, 0x4b1ba7b6434bacd7ull, 0x1a0111ea397fe69aull};
  int N = atoi(argv[1]);
  int hist[2][64] = {{0}}; int mx[2] = {0, 0};
  for (int t = 0; t < N; t++) {
    uint64_t g0[6]; for (int i = 0; i < 6; i++) g0[i] = xr(); g0[5] &= 0x0fffffffffffffffull; // < 2^380 < p
    if (t < 4) { memset(g0, 0, sizeof g0); g0[0] = t + 1; }  // small edge values
    for (int var = 0; var < 2; var++) {
      big f = {{0}}, g = {{0}}; for (int i = 0; i < 6; i++) f.w[i] = (int64_t)P[i], g.w[i] = (int64_t)g0[i];
      int zeta = -1, it = 0;
      while (!iszero(&g)) {
        for (int s = 0; s < 30; s++) {
          int swap = zeta < 0 && (g.w[0] & 1);
          if (swap) { big t2 = g; sub(&g, &f); f = t2; }   // g - f, f <- g
          else if (g.w[0] & 1) add(&g, &f);
          shr1(&g);
          if (var == 0) zeta = swap ? -zeta - 1 : zeta - 1;   // original: zeta = -delta
          else zeta = swap ? -zeta - 2 : zeta - 1;            // half-delta: zeta = -(delta + 1/2)
        }
        it++;
        if (it > 60) { printf("no convergence\n"); return 1; }
      }
      hist[var][it]++; if (it > mx[var]) mx[var] = it;
    }
  }
  for (int var = 0; var < 2; var++) { printf("%s max %d:", var ? "half-delta" : "original", mx[var]); for (int i = 0; i < 64; i++) if (hist[var][i]) printf(" %d:%d", i, hist[var][i]); printf("\n"); }
  return 0;
}
