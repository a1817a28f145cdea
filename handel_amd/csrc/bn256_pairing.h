// bn256_pairing.h — the team Miller loop and final exponentiation shared by
// the pairing kernels (k_verify in bn256_verify.hip; k_pair and the Fp12 probe
// in bn256_pair.hip). One 16-lane team per pairing check (bn256_team.h).
#pragma once
#include "bn256_kernels.h"
#include "bn256_g2team.h"
#include "bn256_xprog.h"

namespace hg {

// ------------------------------------------------------------------ diagnostics
// Built only with -DHG_DIAG (tools/diag.py builds a separate library): lane 0
// of every block accumulates s_memtime cycles per phase of k_verify.
#if defined(HG_DIAG) && defined(HG_DIAG_TU)
__shared__ uint64_t hg_diag_acc[16];
extern __device__ uint64_t g_diag[4096 * 16];
#define DIAG_T0() uint64_t diag_t0_ = __builtin_amdgcn_s_memtime()
#define DIAG_ADD(k)                                                     \
  do {                                                                  \
    uint64_t diag_t1_ = __builtin_amdgcn_s_memtime();                   \
    if (threadIdx.x == 0) hg_diag_acc[k] += diag_t1_ - diag_t0_;        \
    diag_t0_ = diag_t1_;                                                \
  } while (0)
#else
#define DIAG_T0() (void)0
#define DIAG_ADD(k) (void)0
#endif

// ------------------------------------------------------------------ team Miller loop + final exp
// LDS layout per team: 12 Fp12 slots followed by the per-check constants.
static constexpr int kTeamWords = kSlots * kFp12Words + kG2Regs * 10;
static constexpr int kTeamsPerBlock = 4;

// the pairing's final exponentiation (x/crypto optate.go finalExponentiation);
// every program call names the program that follows it (table prefetch, bn256_xprog.h)
HG_DEV void team_final_exp(const Team& T, uint32_t* F, XStream& S) {
  DIAG_T0();
  t12_inv_x<S_A, S_F, S_K, S_L>(T, S, xh<IMul12<S_F, S_B, S_A>>());  // A = f^-1
  DIAG_ADD(5);
  t12_conj(T, S_B, S_F);                                        // B = conj(f)
  x_mul12<S_F, S_B, S_A>(T, S, xh<IMul12<S_F, S_F, S_A>>());   // t1 = f^(p^6 - 1)
  t12_frob2(T, S_A, S_F);
  x_mul12<S_F, S_F, S_A>(T, S, xh<IMul12<S_A, S_A, S_B>>());   // t1 = t1^(p^2 + 1)
  t12_frob(T, S_A, S_F);                                        // fp
  t12_frob2(T, S_B, S_F);                                       // fp2
  x_mul12<S_A, S_A, S_B>(T, S, xh<IMul12<S_A, S_A, S_B>>());
  t12_frob(T, S_B, S_B);                                        // fp3
  x_mul12<S_A, S_A, S_B>(T, S, xh<ICyc<S_J, S_I>>());          // y0 = fp * fp2 * fp3
  DIAG_ADD(6);
  // fu, fu2, fu3 = t1^u, t1^(u^2), t1^(u^3) as nine exponentiations by v
  // (u = v^3) ping-ponging between slots I and J: one copy of the program in
  // the code, run nine times
  t12_copy(T, S_I, S_F);
#pragma unroll 1
  for (int st = 0; st < 9; st++) {
    const XHint next = st == 8 ? xh<IMul12<S_H, S_C, S_H>>() : (st & 1) ? xh<ICyc<S_J, S_I>>() : xh<ICyc<S_I, S_J>>();
    if ((st & 1) == 0) t12_pow_v_x<S_J, S_I>(T, S, next);
    else t12_pow_v_x<S_I, S_J>(T, S, next);
    if (st == 2) t12_copy(T, S_C, S_J);  // fu
    if (st == 5) t12_copy(T, S_D, S_I);  // fu2
    if (st == 8) t12_copy(T, S_E, S_J);  // fu3
  }
  DIAG_ADD(7);
  t12_frob(T, S_G, S_C);
  t12_conj(T, S_G, S_G);                                        // y3 = conj(frob(fu))
  t12_frob(T, S_H, S_D);
  x_mul12<S_H, S_C, S_H>(T, S, xh<IMul12<S_I, S_E, S_I>>());
  t12_conj(T, S_H, S_H);                                        // y4 = conj(fu * frob(fu2))
  t12_frob2(T, S_C, S_D);                                       // y2 = frob2(fu2)
  t12_conj(T, S_D, S_D);                                        // y5 = conj(fu2)
  t12_frob(T, S_I, S_E);
  x_mul12<S_I, S_E, S_I>(T, S, xh<ICyc<S_K, S_I>>());
  t12_conj(T, S_I, S_I);                                        // y6 = conj(fu3 * frob(fu3))
  x_cyc_sqr<S_K, S_I>(T, S, xh<IMul12<S_K, S_K, S_H>>());
  x_mul12<S_K, S_K, S_H>(T, S, xh<IMul12<S_K, S_K, S_D>>());
  x_mul12<S_K, S_K, S_D>(T, S, xh<IMul12<S_J, S_G, S_D>>());   // t0 = y6^2 y4 y5
  x_mul12<S_J, S_G, S_D>(T, S, xh<IMul12<S_J, S_J, S_K>>());
  x_mul12<S_J, S_J, S_K>(T, S, xh<IMul12<S_K, S_K, S_C>>());   // t1 = y3 y5 t0
  x_mul12<S_K, S_K, S_C>(T, S, xh<ICyc<S_J, S_J>>());          // t0 = t0 y2
  x_cyc_sqr<S_J, S_J>(T, S, xh<IMul12<S_J, S_J, S_K>>());
  x_mul12<S_J, S_J, S_K>(T, S, xh<ICyc<S_J, S_J>>());
  x_cyc_sqr<S_J, S_J>(T, S, xh<IMul12<S_K, S_J, S_L>>());      // t1 = (t1^2 t0)^2
  t12_conj(T, S_L, S_F);                                        // y1 = conj(t1_easy)
  x_mul12<S_K, S_J, S_L>(T, S, xh<IMul12<S_J, S_J, S_A>>());   // t0 = t1 y1
  x_mul12<S_J, S_J, S_A>(T, S, xh<ICyc<S_K, S_K>>());          // t1 = t1 y0
  x_cyc_sqr<S_K, S_K>(T, S, xh<IMul12<S_F, S_K, S_J>>());
  x_mul12<S_F, S_K, S_J>(T, S, xh_none());                      // result
  DIAG_ADD(6);
}
// The easy part (f^((p^6 - 1)(p^2 + 1))) of both final exponentiations: the
// result in slot F. h: the program after it.
HG_DEV void team_final_exp_easy(const Team& T, XStream& S, XHint h) {
  t12_inv_x<S_A, S_F, S_K, S_L>(T, S, xh<IMul12<S_F, S_B, S_A>>());  // A = f^-1
  t12_conj(T, S_B, S_F);                                        // B = conj(f)
  x_mul12<S_F, S_B, S_A>(T, S, xh<IMul12<S_F, S_F, S_A>>());   // t1 = f^(p^6 - 1)
  t12_frob2(T, S_A, S_F);
  x_mul12<S_F, S_F, S_A>(T, S, h);                              // t1 = t1^(p^2 + 1)
}

// FE(f)^m with m = 2u(6u^2 + 3u + 1), coprime to r: the hard part of
// Fuentes-Castaneda, Knapp and Rodriguez-Henriquez ("Faster hashing to G2",
// SAC 2011, the BN chain of Duquesne-Ghammam eprint 2015/192 as gnark's bn254
// runs it): three exponentiations by u, 10 multiplications and 3 cyclotomic
// squarings instead of x/crypto's 13 and 4. x -> x^m is a bijection of the
// order-r group GT, so equalities and "== 1" tests of FE values are the same
// with either chain, as long as both sides use this one: k_gt_keys (the GT
// tables), k_verify_sig and k_verify. k_pair and the Fp12 probe keep
// x/crypto's chain (team_final_exp), whose values are compared byte for byte
// with the reference's GT marshal. Oracle: bn256_oracle.final_exponentiation_fc.
//
// The three exponentiations share one copy of the exp-by-v loop (I <-> J,
// base in I, result in J); phase ph prepares the next base between them.
// Slots: F = res, A = t0, B = t1, C = t2, D = t3, E = t4, G scratch, K = the
// exp-by-v scratch. Every input of a hand-written helper (conj, frob, copy)
// is a MUL12 result (canonical); the one squaring that feeds an
// exponentiation's conj is the canonical CYC_SQR program.
HG_DEV void team_final_exp_fc(const Team& T, uint32_t* F, XStream& S) {
  DIAG_T0();
  team_final_exp_easy(T, S, xh<ICyc<S_J, S_I>>());
  DIAG_ADD(5);
  t12_copy(T, S_I, S_F);  // base of the first exponentiation: res
#pragma unroll 1
  for (int ph = 0; ph < 3; ph++) {
#pragma unroll 1
    for (int st = 0; st < 3; st++) {  // J = I^v, I = J^v, J = I^v
      const XHint next = st < 2 ? ((st & 1) ? xh<ICyc<S_J, S_I>>() : xh<ICyc<S_I, S_J>>())
                                : (ph == 0 ? xh<ICyc<S_A, S_A>>() : ph == 1 ? xh<IMul12<S_B, S_C, S_D>>()
                                                                            : xh<IMul12<S_E, S_B, S_J>>());
      if ((st & 1) == 0) t12_pow_v_x<S_J, S_I>(T, S, next);
      else t12_pow_v_x<S_I, S_J>(T, S, next);
    }
    if (ph == 0) {  // t0 = conj(res^u)^2, t1 = t0^2 t0; next base t1
      t12_conj(T, S_A, S_J);
      x_cyc_sqr<S_A, S_A>(T, S, xh<ICyc<S_B, S_A>>());
      x_cyc_sqr<S_B, S_A>(T, S, xh<IMul12<S_B, S_A, S_B>>());
      x_mul12<S_B, S_A, S_B>(T, S, xh<ICyc<S_J, S_I>>());
      t12_copy(T, S_I, S_B);
    } else if (ph == 1) {  // t2 = conj(t1^u), t1 = t2 conj(t1); next base t3 = t2^2
      t12_conj(T, S_C, S_J);
      t12_conj(T, S_D, S_B);
      x_mul12<S_B, S_C, S_D>(T, S, xh<ICyc0<S_I, S_C>>());
      ICyc0<S_I, S_C>::run(T, S, xh<ICyc<S_J, S_I>>());
    } else {  // t4 = t1 t3^u
      x_mul12<S_E, S_B, S_J>(T, S, xh<IMul12<S_D, S_A, S_E>>());
    }
  }
  DIAG_ADD(7);
  x_mul12<S_D, S_A, S_E>(T, S, xh<IMul12<S_A, S_C, S_E>>());  // t3 = t0 t4
  x_mul12<S_A, S_C, S_E>(T, S, xh<IMul12<S_A, S_F, S_A>>());  // t0 = t2 t4
  x_mul12<S_A, S_F, S_A>(T, S, xh<IMul12<S_A, S_G, S_A>>());  // t0 = res t0
  t12_frob(T, S_G, S_D);
  x_mul12<S_A, S_G, S_A>(T, S, xh<IMul12<S_A, S_G, S_A>>());  // t0 = frob(t3) t0
  t12_frob2(T, S_G, S_E);
  x_mul12<S_A, S_G, S_A>(T, S, xh<IMul12<S_G, S_G, S_D>>());  // t0 = frob2(t4) t0
  t12_conj(T, S_G, S_F);
  x_mul12<S_G, S_G, S_D>(T, S, xh<IMul12<S_F, S_G, S_A>>());  // t2 = conj(res) t3
  t12_frob(T, S_G, S_G);
  t12_frob2(T, S_G, S_G);                                       // t2 = frob^3(t2)
  x_mul12<S_F, S_G, S_A>(T, S, xh_none());                      // result
  DIAG_ADD(6);
}

// the first program team_final_exp runs (t12_inv_x<S_A, S_F, S_K, S_L>)
HG_DEV constexpr XHint final_exp_hint() { return xh<IMul12<S_L, S_F, S_K>>(); }

// Per-check inputs of the team Miller loop.
struct CheckCtx {
  Fp2 qx, qy;   // affine pk (a dummy valid point when the pk is infinity)
  Fp hx, hy;    // H (affine)
  Fp sx, sy;    // sig (affine)
  bool use_q;   // pk contributes (not infinity)
  bool use_s;   // sig contributes (not infinity)
};

// Writes the team's G2 register file: point R = Q (projective, see below), Q, -Qy, the
// Frobenius images q1 = pi(Q), -q2 = (Qx gamma2[2], Qy) (optate.go miller),
// the G1 points and constants. has_fixed && C.use_s: the G2Base pairing at
// -sig contributes; otherwise SX = NSY = 0 make every evaluated G2Base line
// w^3, an element of Fp4 that the final exponentiation maps to 1 (x/crypto's
// GT = 1 for an infinity input).
HG_DEV void g2_regs_init(const Team& T, uint32_t* F, const CheckCtx& C, bool has_fixed) {
  const Fp2 g1[6] = HG_GAMMA1;
  const Fp g2[6] = HG_GAMMA2;
  Fp2 nqy, q1x, q1y, q2x, t, one2;
  f2_neg(nqy, C.qy);
  f2_conj(t, C.qx);
  f2_mul(q1x, t, g1[2]);
  f2_conj(t, C.qy);
  f2_mul(q1y, t, g1[3]);
  f2_muls(q2x, C.qx, g2[2]);
  f2_one(one2);
  Fp zero, one, nsy;
  fp_zero(zero);
  fp_one(one);
  fp_neg(nsy, C.sy);
  if (T.tl == 0) {
    auto put2 = [&](int rx, const Fp2& v) {
      st_fp(F + rx * 10, v.x);
      st_fp(F + (rx + 1) * 10, v.y);
    };
    st_fp(F + R_ZERO * 10, zero);
    st_fp(F + R_ONE * 10, one);
    st_fp(F + R_PX * 10, C.hx);
    st_fp(F + R_PY * 10, C.hy);
    const bool fix = has_fixed && C.use_s;
    st_fp(F + R_SX * 10, fix ? C.sx : zero);
    st_fp(F + R_NSY * 10, fix ? nsy : zero);
    // R = (xi Qx : xi Qy : xi) in the projective programs' coordinates, whose
    // Z register holds W = Z / xi = 1 (gen_g2_schedule.py prog_double_proj)
    Fp2 xqx, xqy;
    f2_mul_xi(xqx, C.qx);
    f2_mul_xi(xqy, C.qy);
    put2(R_X_x, xqx);
    put2(R_Y_x, xqy);
    put2(R_Z_x, one2);
    put2(R_QX_x, C.qx);
    put2(R_QY_x, C.qy);
    put2(R_NQY_x, nqy);
    put2(R_P1X_x, q1x);
    put2(R_P1Y_x, q1y);
    put2(R_P2X_x, q2x);
  }
  team_sync();
}

// The normalised G2Base line (bx, cy: 4 Fp; a = 1, k_g2_lines) goes into FBX,
// FCY from one VGPR element per lane (lane tl < 4 holds Fp tl), read from the
// table one line ahead so the L2 latency of the read overlaps the step's rounds.
HG_DEV void fixed_line_fetch(const Team& T, Fp& held, const LineCoef* tab, int s) {
  if (T.tl < 4 && s < kNumLines) held = reinterpret_cast<const Fp*>(&tab[s])[T.tl];
}
// publishes the held line, then fetches line `next`
HG_DEV void load_fixed_line(const Team& T, uint32_t* F, Fp& held, const LineCoef* tab, int next) {
  if (T.tl < 4) st_fp(F + (R_FBX_x + T.tl) * 10, held);
  team_sync();
  fixed_line_fetch(T, held, tab, next);
}

// A pk at infinity contributes the unit line (a = b = 0, c = 1): the pk line
// (LA, LB, LC) is replaced before x_line_pk; the branch is taken only when
// some team of the wave needs it. The G2Base side needs no replacement
// (g2_regs_init).
HG_DEV void unit_line_regs(const Team& T, uint32_t* F, bool fix, int ra, int rb, int rc) {
  if (__ballot(fix) == 0) return;  // wave-uniform
  Fp z, o;
  fp_zero(z);
  fp_one(o);
  if (T.tl < 6 && fix) {
    // element tl of (a.x, a.y, b.x, b.y, c.x, c.y); c.y is the real part of c
    Fp v;
    fp_sel(v, T.tl == 5, o, z);
    const int r = T.tl < 2 ? ra + T.tl : (T.tl < 4 ? rb + T.tl - 2 : rc + T.tl - 4);
    st_fp(F + r * 10, v);
  }
  team_sync();
}
HG_DEV void unit_line_pk(const Team& T, uint32_t* F, const CheckCtx& C) {
  unit_line_regs(T, F, !C.use_q, R_LA_x, R_LB_x, R_LC_x);
}

// The Miller loop's fused programs (gen_g2_schedule.py FUSED): a doubling step
// is MDBL_1 (f^2 beside the doubling's first round), MDBL_2 (f * G2Base line
// beside its second round) and the pk line; an addition step is PADD_*_1,
// MADD_*_2 (f * G2Base line beside the second round), PADD_*_3, pk line.
template <int P1, int P2, int P3>
struct AddStep {
  using I1 = XInst<P1>;
  using I2 = XInst<P2, S_F, S_F>;
  using I3 = XInst<P3>;
};
// ... bound to a team region: the full layout (MillerFull: k_verify,
// k_gt_keys, k_pair) or layout V (MillerV: k_verify_ml, the Miller loop alone)
struct MillerFull {
  using Mdbl1 = XInst<XP_MDBL_1, S_F, S_F>;
  using Mdbl2 = XInst<XP_MDBL_2, S_F, S_F>;
  using Pdbl1 = XInst<XP_PDBL_1>;
  using LinePk = XInst<XP_LINE_PK, S_F, S_F>;
  using AddPos = AddStep<XP_PADD_POS_1, XP_MADD_POS_2, XP_PADD_POS_3>;
  using AddNeg = AddStep<XP_PADD_NEG_1, XP_MADD_NEG_2, XP_PADD_NEG_3>;
  using AddF1 = AddStep<XP_PADD_F1_1, XP_MADD_F1_2, XP_PADD_F1_3>;
  using AddF2 = AddStep<XP_PADD_F2_1, XP_MADD_F2_2, XP_PADD_F2_3>;
};
struct MillerV {
  using Mdbl1 = XInst<XP_MDBL_1_V, S_F, S_F>;
  using Mdbl2 = XInst<XP_MDBL_2_V, S_F, S_F>;
  using Pdbl1 = XInst<XP_PDBL_1_V>;
  using LinePk = XInst<XP_LINE_PK_V, S_F, S_F>;
  using AddPos = AddStep<XP_PADD_POS_1_V, XP_MADD_POS_2_V, XP_PADD_POS_3_V>;
  using AddNeg = AddStep<XP_PADD_NEG_1_V, XP_MADD_NEG_2_V, XP_PADD_NEG_3_V>;
  using AddF1 = AddStep<XP_PADD_F1_1_V, XP_MADD_F1_2_V, XP_PADD_F1_3_V>;
  using AddF2 = AddStep<XP_PADD_F2_1_V, XP_MADD_F2_2_V, XP_PADD_F2_3_V>;
};

template <class L, class A>
HG_DEV void add_step(const Team& T, uint32_t* F, const CheckCtx& C, XStream& S, XHint next) {
  A::I1::run(T, S, xh<typename A::I2>());
  A::I2::run(T, S, xh<typename A::I3>());
  A::I3::run(T, S, xh<typename L::LinePk>());
  unit_line_pk(T, F, C);
  L::LinePk::run(T, S, next);
}

// f = Miller(pk at H) * Miller(G2Base at -sig) (x/crypto optate.go miller, with
// the two loops sharing their squarings); the G2 steps run as team programs.
// after: the program that runs after the loop.
template <class L = MillerFull>
HG_DEV void team_miller_check(const Team& T, uint32_t* F, const CheckCtx& C, const LineCoef* tab, bool has_fixed,
                              XStream& S, XHint after) {
  using IMdbl1 = typename L::Mdbl1;
  using IMdbl2 = typename L::Mdbl2;
  using AddPos = typename L::AddPos;
  using AddNeg = typename L::AddNeg;
  using AddF1 = typename L::AddF1;
  using AddF2 = typename L::AddF2;
  const int8_t naf[kNafLen] = HG_NAF;
  constexpr XHint kLinePk = xh<typename L::LinePk>();
  t12_set_one(T, S_F);
  g2_regs_init(T, F, C, has_fixed);
  Fp held;
  fp_zero(held);
  fixed_line_fetch(T, held, tab, 0);
  int s = 0;
  DIAG_T0();
  for (int i = kNafLen - 1; i > 0; i--) {
    load_fixed_line(T, F, held, tab, ++s);
    DIAG_ADD(0);
    if (i == kNafLen - 1) L::Pdbl1::run(T, S, xh<IMdbl2>());  // f = 1: no squaring
    else IMdbl1::run(T, S, xh<IMdbl2>());
    DIAG_ADD(1);
    IMdbl2::run(T, S, kLinePk);
    unit_line_pk(T, F, C);
    DIAG_ADD(2);
    const int d = naf[i - 1];
    const XHint step = i > 1 ? xh<IMdbl1>() : xh<typename AddF1::I1>();  // after this digit
    L::LinePk::run(T, S, d > 0 ? xh<typename AddPos::I1>() : d < 0 ? xh<typename AddNeg::I1>() : step);
    DIAG_ADD(3);
    if (d != 0) {
      load_fixed_line(T, F, held, tab, ++s);
      DIAG_ADD(0);
      if (d > 0) add_step<L, AddPos>(T, F, C, S, step);
      else add_step<L, AddNeg>(T, F, C, S, step);
      DIAG_ADD(4);
    }
  }
  load_fixed_line(T, F, held, tab, ++s);
  add_step<L, AddF1>(T, F, C, S, xh<typename AddF2::I1>());
  load_fixed_line(T, F, held, tab, ++s);
  add_step<L, AddF2>(T, F, C, S, after);
}

HG_DEV uint32_t* team_regs(const Team& T) { return T.base + kSlots * kFp12Words; }

}  // namespace hg
