/*
 * C caller of include/cess_bls.h (test infrastructure): compiled by gcc as
 * C99 with -Wall -Wextra -Werror -pedantic, so the header is checked by a C
 * compiler and not only through ctypes.
 *
 * Input: a text file of golden records (tests/golden/vectors.json, written out
 * by tests/test_c_abi.py), one per line: "<sig hex> <msg hex> <pk hex> <code>"
 * ("-" for an empty field).  The program verifies every record through
 * cess_bls_verify_batch_var, cess_bls_verify (one by one) and, when every
 * record has fixed lengths, cess_bls_verify_batch, and compares codes and the
 * bitmap with the expected codes.
 *
 * Exit status: 0 all equal; 1 mismatch; 2 no HIP device (ctx_create returned
 * CESS_BLS_E_NO_DEVICE, the expected outcome on a machine without a GPU);
 * 3 usage / input / infrastructure error.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "cess_bls.h"

typedef struct {
  uint8_t* b;
  size_t n, cap;
} buf;

static void put(buf* d, const uint8_t* p, size_t n) {
  if (d->n + n > d->cap) {
    d->cap = 2 * (d->n + n) + 64;
    d->b = (uint8_t*)realloc(d->b, d->cap);
    if (!d->b) exit(3);
  }
  if (n) memcpy(d->b + d->n, p, n);
  d->n += n;
}

static int hexval(int c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  return -1;
}

/* append the bytes of a hex token to d; returns the byte count or -1 */
static long unhex(const char* s, buf* d) {
  size_t len = strlen(s), i;
  if (strcmp(s, "-") == 0) return 0;
  if (len % 2) return -1;
  for (i = 0; i < len; i += 2) {
    int hi = hexval(s[i]), lo = hexval(s[i + 1]);
    uint8_t v;
    if (hi < 0 || lo < 0) return -1;
    v = (uint8_t)(hi * 16 + lo);
    put(d, &v, 1);
  }
  return (long)(len / 2);
}

int main(int argc, char** argv) {
  FILE* f;
  char line[8192];
  buf sigs = {0}, msgs = {0}, pks = {0};
  uint64_t *so, *mo, *po;
  uint8_t *expect, *codes;
  uint64_t* bitmap;
  size_t n = 0, cap = 1024, i;
  int fixed = 1, bad = 0, st;
  cess_bls_config cfg;
  cess_bls_ctx* ctx = NULL;

  if (argc != 2) return 3;
  f = fopen(argv[1], "r");
  if (!f) return 3;
  so = (uint64_t*)calloc(cap + 1, 8);
  mo = (uint64_t*)calloc(cap + 1, 8);
  po = (uint64_t*)calloc(cap + 1, 8);
  expect = (uint8_t*)calloc(cap, 1);
  if (!so || !mo || !po || !expect) return 3;
  while (fgets(line, sizeof line, f)) {
    char s[512], m[4096], p[512];
    int code;
    long ls, lm, lp;
    if (sscanf(line, "%511s %4095s %511s %d", s, m, p, &code) != 4) continue;
    if (n == cap) return 3;
    ls = unhex(s, &sigs);
    lm = unhex(m, &msgs);
    lp = unhex(p, &pks);
    if (ls < 0 || lm < 0 || lp < 0) return 3;
    so[n + 1] = so[n] + (uint64_t)ls;
    mo[n + 1] = mo[n] + (uint64_t)lm;
    po[n + 1] = po[n] + (uint64_t)lp;
    if (ls != CESS_BLS_SIG_BYTES || lp != CESS_BLS_PK_BYTES) fixed = 0;
    expect[n++] = (uint8_t)code;
  }
  fclose(f);
  if (n == 0) return 3;

  memset(&cfg, 0, sizeof cfg);
  cfg.device = 0;
  cfg.max_batch = 4096;
  st = cess_bls_ctx_create(&cfg, &ctx);
  if (st == CESS_BLS_E_NO_DEVICE) {
    printf("no device: %s\n", cess_bls_status_string(st));
    return 2;
  }
  if (st != CESS_BLS_OK) {
    printf("ctx_create: %s\n", cess_bls_status_string(st));
    return 3;
  }
  codes = (uint8_t*)calloc(n, 1);
  bitmap = (uint64_t*)calloc((n + 63) / 64, 8);
  if (!codes || !bitmap) return 3;

  st = cess_bls_verify_batch_var(ctx, n, sigs.b, so, pks.b, po, msgs.b, mo, codes, bitmap);
  if (st != CESS_BLS_OK) {
    printf("verify_batch_var: %s\n", cess_bls_status_string(st));
    return 3;
  }
  for (i = 0; i < n; i++) {
    int bit = (int)((bitmap[i / 64] >> (i % 64)) & 1u);
    if (codes[i] != expect[i] || bit != (expect[i] == CESS_BLS_CODE_OK)) {
      printf("batch_var record %zu: code %d expected %d bit %d\n", i, codes[i], expect[i], bit);
      bad++;
    }
  }
  for (i = 0; i < n; i++) {
    uint8_t c = 0xff;
    st = cess_bls_verify(ctx, sigs.b + so[i], (size_t)(so[i + 1] - so[i]), msgs.b ? msgs.b + mo[i] : NULL,
                         (size_t)(mo[i + 1] - mo[i]), pks.b + po[i], (size_t)(po[i + 1] - po[i]), &c);
    if (st != CESS_BLS_OK || c != expect[i]) {
      printf("verify record %zu: status %d code %d expected %d\n", i, st, c, expect[i]);
      bad++;
    }
  }
  if (fixed) {
    memset(codes, 0xff, n);
    st = cess_bls_verify_batch(ctx, n, sigs.b, pks.b, msgs.b, mo, codes, NULL);
    if (st != CESS_BLS_OK) return 3;
    for (i = 0; i < n; i++)
      if (codes[i] != expect[i]) {
        printf("batch record %zu: code %d expected %d\n", i, codes[i], expect[i]);
        bad++;
      }
  }
  cess_bls_ctx_destroy(ctx);
  printf("%s: %zu records, %d mismatches (%s)\n", bad ? "FAIL" : "OK", n, bad, cess_bls_version());
  return bad ? 1 : 0;
}
