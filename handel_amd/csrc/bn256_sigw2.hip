// bn256_sigw2.hip — the latency form of the GT path's signature pairing:
// k_verify_sig<4, true>'s program with each 16-lane team spread over the two
// waves of a workgroup. This translation unit alone enables
// split teams (HG_TEAM_SPLIT, bn256_team.h), so the one-wave kernels of every
// other unit compile without the split branches.
#define HG_TEAM_SPLIT 1
#include <hip/hip_runtime.h>

#include "bn256_decode.h"
#include "bn256_gt.h"
#include "bn256_sigteam.h"

namespace hg {
static inline int nblk(int n, int b) { return (n + b - 1) / b; }

// The latency form of k_verify_sig<4, true>: each 16-lane team spans the two
// waves of a 128-thread workgroup (make_team_w2), which split every round's
// products between them (bn256_xprog.h x_job_split), so a check's dependent
// chain is about half as long for the same values. Twice the waves per check:
// it pays when the batch is small (n <= kSigW2MaxN: 2n waves still fit one per
// SIMD) and the step waits on the pairing — a lone batch's latency.
__global__ __launch_bounds__(128) void k_verify_sig_w2(const uint8_t* sig_bytes, int flavor, int n,
                                                       const LineCoef* tab, Gt* fe) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[4 * kSigTeamWords + 4 * 16 * kXchgWords];
  __builtin_amdgcn_s_setprio(3);
  // one wave per SIMD: a workgroup's two waves on two SIMDs of the CU
  asm volatile("" ::: "v255", "a0");
  Team T = make_team_w2(lds, kSigTeamWords, lds + 4 * kSigTeamWords);
  uint32_t* F = T.base + kSigRegBase * 10;
  const int idx = blockIdx.x * 4 + ((threadIdx.x & 63) >> 4);
  const bool valid = idx < n;
  const int ci = valid ? idx : n - 1;
  PointG1 sg;
  (void)decode_g1_one(sig_bytes + (size_t)ci * 64, flavor, sg);
  XStream S = x_stream();
  team_miller_sig(T, F, sg.x, sg.y, sg.inf == 0, tab, S, SigFE<SigProgs16>::final_exp_hint_s());
  SigFE<SigProgs16>::team_final_exp_fc_s(T, S);
  team_sync(T);
  if (valid && T.wave == 0) gt_store(T, S_F, fe + idx);
}

void launch_sig_pairing_w2(const uint8_t* sigs, int flavor, int n, const LineCoef* tab, Gt* fe, hipStream_t s) {
  if (n > 0) k_verify_sig_w2<<<nblk(n, 4), 128, 0, s>>>(sigs, flavor, n, tab, fe);
}
}  // namespace hg
