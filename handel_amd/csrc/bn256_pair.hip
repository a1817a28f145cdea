// bn256_pair.hip — k_pair (bn256.Pair(g1, g2).Marshal(), the GT parity probe)
// and k_fp12_op (team Fp12 building blocks for the parity tests).
#include <hip/hip_runtime.h>

#include "bn256_pairing.h"

namespace hg {
static inline int nblk(int n, int b) { return (n + b - 1) / b; }

// bn256.Pair(g1, g2).Marshal() for n pairs (GT = 1 when either is infinity)
__global__ __launch_bounds__(64) void k_pair(const PointG1* g1s, const PointG2* g2s, int n, const LineCoef* tab,
                                             uint8_t* gt_out) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[kTeamsPerBlock * kTeamWords];
  Team T = make_team(lds, kTeamWords);
  uint32_t* F = team_regs(T);
  int idx = blockIdx.x * kTeamsPerBlock + (threadIdx.x >> 4);
  bool valid = idx < n;
  int ci = valid ? idx : n - 1;
  PointG1 P = g1s[ci];
  PointG2 Q = g2s[ci];
  CheckCtx C;
  C.use_q = (P.inf == 0) && (Q.inf == 0);
  C.use_s = false;
  if (!C.use_q) {
    const Fp2 gx = HG_G2X, gy = HG_G2Y;
    Q.x = gx;
    Q.y = gy;
    const Fp hx = HG_G1X, hy = HG_G1Y;
    P.x = hx;
    P.y = hy;
  }
  C.qx = Q.x;
  C.qy = Q.y;
  C.hx = P.x;
  C.hy = P.y;
  fp_zero(C.sx);
  fp_zero(C.sy);
  XStream S = x_stream();
  team_miller_check(T, F, C, tab, false, S, final_exp_hint());
  team_final_exp(T, F, S);  // f == 1 when either input is infinity, and 1^e == 1
  // GT.Marshal order: coefficients 5,3,1,4,2,0, each as (x, y)
  if (valid && T.active) {
    const int pos[6] = {5, 2, 4, 1, 3, 0};  // position of coefficient k in the marshal
    Fp v;
    ld_fp(v, slot(T, S_F) + T.e * 10);
    // comp 0 (x) first, comp 1 (y) second
    uint8_t* o = gt_out + (size_t)idx * 384 + pos[T.k] * 64 + (T.comp ? 32 : 0);
    fp_to_be(o, v);
  }
}

// Team Fp12 op probe (parity tests of the building blocks): inputs/outputs are
// 384-byte GT-marshal-ordered canonical elements.
//   op 0 a*b, 1 a^2 (merged products), 2 cyclotomic a^2, 3 a^p, 4 a^(p^2),
//   5 a^-1, 6 conj(a), 7 a^u (cyclotomic), 8 final exponentiation
__global__ __launch_bounds__(64) void k_fp12_op(int op, const uint8_t* a, const uint8_t* b, int n, uint8_t* out) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[kTeamsPerBlock * kTeamWords];
  Team T = make_team(lds, kTeamWords);
  uint32_t* F = T.base + kSlots * kFp12Words;
  int idx = blockIdx.x * kTeamsPerBlock + (threadIdx.x >> 4);
  bool valid = idx < n;
  int ci = valid ? idx : n - 1;
  const int pos[6] = {5, 2, 4, 1, 3, 0};
  if (T.active) {
    Fp v;
    bool ge;
    fp_from_be(v, a + (size_t)ci * 384 + pos[T.k] * 64 + (T.comp ? 32 : 0), &ge);
    st_fp(slot(T, S_A) + T.e * 10, v);
    fp_from_be(v, b + (size_t)ci * 384 + pos[T.k] * 64 + (T.comp ? 32 : 0), &ge);
    st_fp(slot(T, S_B) + T.e * 10, v);
  }
  team_sync();
  {
    Fp z, one;
    fp_zero(z);
    fp_one(one);
    if (T.tl == 0) {
      st_fp(F + R_ZERO * 10, z);
      st_fp(F + R_ONE * 10, one);
    }
    team_sync();
  }
  // op bits 8..: repetitions (timing of one building block: reps - 1 extra
  // applications feed the result back as the input)
  int reps = (op >> 8) > 0 ? (op >> 8) : 1;
  op &= 255;
  XStream S = x_stream();
  for (int r = 0; r < reps; r++) {
    if (r > 0) t12_copy(T, S_A, S_F);
    switch (op) {  // kernel-uniform
      case 0: x_mul12<S_F, S_A, S_B>(T, S, xh_none()); break;
      case 1: x_sqr12<S_F, S_A>(T, S, xh_none()); break;
      case 2: x_cyc_sqr<S_F, S_A>(T, S, xh_none()); break;
      case 3: t12_frob(T, S_F, S_A); break;
      case 4: t12_frob2(T, S_F, S_A); break;
      case 5: t12_inv_x<S_F, S_A, S_K, S_L>(T, S, xh_none()); break;
      case 6: t12_conj(T, S_F, S_A); break;
      case 7: t12_pow_u_x<S_F, S_A>(T, S, xh_none()); break;
      case 8: t12_copy(T, S_F, S_A); team_final_exp(T, F, S); break;
      case 9: t12_sqr_fast(T, S_F, S_A); break;
      case 10: t12_cyc_sqr(T, S_F, S_A); break;
      default: t12_copy(T, S_F, S_A); break;
    }
  }
  if (valid && T.active) {
    Fp v;
    ld_fp(v, slot(T, S_F) + T.e * 10);
    fp_to_be(out + (size_t)idx * 384 + pos[T.k] * 64 + (T.comp ? 32 : 0), v);
  }
}

void launch_pair(const PointG1* g1s, const PointG2* g2s, int n, const LineCoef* tab, uint8_t* gt, hipStream_t s) {
  if (n > 0) k_pair<<<nblk(n, kTeamsPerBlock), 64, 0, s>>>(g1s, g2s, n, tab, gt);
}
void launch_fp12_op(int op, const uint8_t* a, const uint8_t* b, int n, uint8_t* out, hipStream_t s) {
  if (n > 0) k_fp12_op<<<nblk(n, kTeamsPerBlock), 64, 0, s>>>(op, a, b, n, out);
}
}  // namespace hg
