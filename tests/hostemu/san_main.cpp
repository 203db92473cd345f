// TEST HARNESS ONLY: sanitizer driver for the host-emulation build (the
// device headers compiled for the host, tests/hostemu/emu.cpp).  Built by
// tests/test_sanitizers.py with -fsanitize=address,undefined and run on the
// golden records (one per line: "<sig hex> <msg hex> <pk hex> <code>"); any
// sanitizer report aborts the process (halt_on_error), a code mismatch exits 1.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

extern "C" int emu_verify(const uint8_t* sig, const uint8_t* msg, uint32_t mlen, const uint8_t* pk, uint8_t* gt_out);
extern "C" int emu_gt_valuebased(const uint8_t* sig, const uint8_t* msg, uint32_t mlen, const uint8_t* pk,
                                 uint8_t* gt_out);

static std::vector<uint8_t> unhex(const std::string& h) {
  std::vector<uint8_t> b;
  if (h == "-") return b;
  for (size_t i = 0; i + 1 < h.size(); i += 2) b.push_back((uint8_t)strtoul(h.substr(i, 2).c_str(), nullptr, 16));
  return b;
}

int main(int argc, char** argv) {
  if (argc != 2) return 2;
  FILE* f = fopen(argv[1], "r");
  if (!f) return 2;
  char s[256], m[1024], p[512];
  int code, n = 0, bad = 0;
  while (fscanf(f, "%255s %1023s %511s %d", s, m, p, &code) == 4) {
    auto sig = unhex(s), msg = unhex(m), pk = unhex(p);
    uint8_t gt[576], gt2[576];
    const int c = emu_verify(sig.data(), msg.data(), (uint32_t)msg.size(), pk.data(), gt);
    if (c != code) {
      printf("record %d: code %d expected %d\n", n, c, code);
      bad++;
    }
    if (c == 0 || c == 5) {   // both pairing paths agree on Gt
      const int c2 = emu_gt_valuebased(sig.data(), msg.data(), (uint32_t)msg.size(), pk.data(), gt2);
      if (c2 != c || memcmp(gt, gt2, 576) != 0) {
        printf("record %d: value-based path differs\n", n);
        bad++;
      }
    }
    n++;
  }
  fclose(f);
  printf("%s: %d records, %d mismatches\n", bad ? "FAIL" : "OK", n, bad);
  return bad ? 1 : 0;
}
