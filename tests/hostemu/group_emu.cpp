// TEST HARNESS ONLY: the lane-group program of the small-batch path
// (cess_amd/csrc/bls/group_prog.hpp) run on the host with the kernel's own
// operation body (bls/group.hpp group_eval, -DCESS_HOSTEMU) and the kernel's
// round semantics (every lane of a round reads before any lane writes), so the
// entry encoding, the Montgomery constants and the lazy-reduction bounds are
// checked against the golden Gt bytes without a GPU.  Never linked into the
// product library.
#include <string.h>

#include <vector>

#include "../../cess_amd/csrc/bls/group.hpp"

using namespace bls;

namespace {
struct HostRegs {
  std::vector<fp2>* S;
  fp2 ld(uint32_t s) const { return (*S)[s]; }
  fp ld_comp(uint32_t s, uint32_t comp) const { return comp ? (*S)[s].c1 : (*S)[s].c0; }
};
fp load_raw(const uint32_t* x) {
  fp r;
  memcpy(r.v, x, 48);
  return r;
}
}  // namespace

extern "C" {
// in: 7 Fp2 in raw canonical limbs (p0x p0y p1x p1y qx qy one), c0 then c1;
// out: 11 Fp2 raw canonical (tx ty tz pzx pzy gt0..gt5); returns the round count
int group_emu_run(const uint32_t* in, uint32_t* out) {
  std::vector<fp2> S(grp::N_SLOTS, fp2_zero());
  const int ins[7] = {grp::IN_P0X, grp::IN_P0Y, grp::IN_P1X, grp::IN_P1Y, grp::IN_QX, grp::IN_QY, grp::IN_ONE};
  for (int k = 0; k < 7; k++) S[ins[k]] = {to_mont(load_raw(in + 24 * k)), to_mont(load_raw(in + 24 * k + 12))};
  HostRegs R{&S};
  // the kernel's lanes: lane 2 op + comp computes component comp of op
  std::vector<std::pair<uint32_t, std::pair<uint32_t, fp>>> wr;
  for (int r = 0; r < grp::N_ROUNDS; r++) {
    const uint32_t h = grp::kRounds[r];
    const uint32_t kind = h & 0xffu, cnt = (h >> 8) & 0xffu, off = h >> 16;
    wr.clear();
    for (uint32_t lane = 0; lane < 2 * cnt; lane++) {
      const uint32_t* e = grp::kEnts[off + (lane >> 1)];
      uint32_t d;
      const fp v = group_eval_comp(R, kind, e[0], e[1], e[2], e[3], lane & 1, &d);
      wr.push_back({d, {lane & 1, v}});
    }
    for (auto& w : wr) (w.second.first ? S[w.first].c1 : S[w.first].c0) = w.second.second;
  }
  const int outs[11] = {grp::OUT_TX,  grp::OUT_TY,  grp::OUT_TZ,  grp::OUT_PZX, grp::OUT_PZY, grp::OUT_GT0,
                        grp::OUT_GT1, grp::OUT_GT2, grp::OUT_GT3, grp::OUT_GT4, grp::OUT_GT5};
  for (int k = 0; k < 11; k++) {
    const fp c0 = from_mont(S[outs[k]].c0), c1 = from_mont(S[outs[k]].c1);
    memcpy(out + 24 * k, c0.v, 48);
    memcpy(out + 24 * k + 12, c1.v, 48);
  }
  return grp::N_ROUNDS;
}
}
