// bn256_sigw2.hip — k_verify_sig_split<2> (bn256_sigsplit.h): a check's 16-lane
// team over 2 waves. This unit alone builds 2-wave split teams
// (HG_TEAM_SPLIT, bn256_team.h), so the one-wave kernels of every other unit
// compile without the split branches.
#define HG_TEAM_SPLIT 2
#include "bn256_sigsplit.h"

namespace hg {

void launch_sig_pairing_w2(const uint8_t* sigs, int flavor, int n, const LineCoef* tab, Gt* fe, hipStream_t s) {
  if (n > 0) k_verify_sig_split<2><<<(n + 3) / 4, 64 * 2, 0, s>>>(sigs, flavor, n, tab, fe);
}

}  // namespace hg
