// bn256_sigsplit.h — the latency forms of the GT path's signature pairing
// (DESIGN.md §3e): k_verify_sig<4, true>'s program on teams spread over NW
// waves. Included only by the units that build split teams (bn256_sigw2.hip:
// HG_TEAM_SPLIT defined before any include). A 4-wave form (same code, a
// unit with HG_TEAM_SPLIT 4) measured slower than the 2-wave one: 0.826 vs
// 0.757 ms for 128 checks (profiles/r05w4_latency.json).
#pragma once

#include <hip/hip_runtime.h>

#include "bn256_decode.h"
#include "bn256_gt.h"
#include "bn256_sigteam.h"

namespace hg {

// The latency forms of k_verify_sig<4, true>: each 16-lane team spans the NW
// waves of a 64 NW-thread workgroup (make_team_split), which split every
// round's products and pre-pass values between them (bn256_xprog.h
// x_job_split), so a check's dependent chain is shorter for the same values.
// NW times the waves per check: it pays when the batch is small (NW n / 4
// waves still fit one per SIMD) and the step waits on the pairing — a lone
// batch's latency. Instantiated only in the unit built with HG_TEAM_SPLIT = NW.
template <int NW>
__global__ __launch_bounds__(64 * NW) void k_verify_sig_split(const uint8_t* sig_bytes, int flavor, int n,
                                                              const LineCoef* tab, Gt* fe) {
  static_assert(NW == kSplitWaves, "built with HG_TEAM_SPLIT = NW");
  __shared__ __attribute__((aligned(16))) uint32_t lds[4 * kSigTeamWords + 4 * 16 * (NW - 1) * kXchgWords];
  __builtin_amdgcn_s_setprio(3);
  // one wave per SIMD: a workgroup's waves on different SIMDs of the CU
  asm volatile("" ::: "v255", "a0");
  Team T = make_team_split(lds, kSigTeamWords, lds + 4 * kSigTeamWords);
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

}  // namespace hg
