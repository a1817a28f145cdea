// bn256_sigteam.h — the pieces of the GT path's signature-side pairing that
// both of its 16-lane kernels use: GT values between HBM and team slots, the
// Miller loop at -sig (G2Base lines from the table), the layout-S team region.
// k_verify_sig (bn256_gt.hip) runs them on one wave per team, the latency form
// k_verify_sig_split (bn256_sigsplit.h) on teams spread over 2 or 4 waves.
#pragma once

#include "bn256_gt.h"
#include "bn256_pairing.h"
#include "bn256_sigfe.h"

namespace hg {

// ------------------------------------------------------------------ GT values in HBM <-> team slots
// A GT value in HBM is the team slot layout: element e (10 limbs) at w[10 e].
// Lane e < 12 moves element e; `conj` negates the odd powers of w on the way
// in (the inverse of a unitary value). No sync: callers sync before reading.
HG_DEV void gt_read(Fp& v, const Gt* g, const Team& T) {
  const uint2* src = (const uint2*)__builtin_assume_aligned(g->w + 10 * T.e, 8);
#pragma unroll
  for (int i = 0; i < 5; i++) {
    const uint2 x = src[i];
    v.l[2 * i] = x.x;
    v.l[2 * i + 1] = x.y;
  }
}
HG_DEV void gt_put(const Team& T, int s, const Fp& v0, bool conj) {
  Fp v = v0;
  if (conj) {
    Fp n;
    fp_neg(n, v);
    fp_sel(v, (T.k & 1) != 0, n, v);
  }
  if (T.active) st_fp_a8(slot(T, s) + T.e * 10, v.l);
}
HG_DEV void gt_load(const Team& T, int s, const Gt* g, bool conj = false) {
  Fp v;
  gt_read(v, g, T);
  gt_put(T, s, v, conj);
}
HG_DEV void gt_one_value(Fp& v, const Team& T) {
  Fp one;
  fp_one(one);
  fp_zero(v);
  fp_sel(v, T.e == 1, one, v);  // element 1 = c0.y
}
// slot s = g (present) or 1
HG_DEV void gt_load_or_one(const Team& T, int s, const Gt* g, bool present) {
  Fp v, one;
  gt_one_value(one, T);
  if (present) gt_read(v, g, T);
  fp_sel(v, present, v, one);
  gt_put(T, s, v, false);
}
HG_DEV void gt_store(const Team& T, int s, Gt* g) {
  Fp v;
  ld_fp_a8(v, slot(T, s) + T.e * 10);
  if (!T.active) return;
  uint2* dst = (uint2*)__builtin_assume_aligned(g->w + 10 * T.e, 8);
#pragma unroll
  for (int i = 0; i < 5; i++) dst[i] = make_uint2(v.l[2 * i], v.l[2 * i + 1]);
}
// element-wise copy between team-region Fp12 values (LDS pointers)
HG_DEV void lds_fp12_copy(const Team& T, uint32_t* dst, const uint32_t* src) {
  Fp v;
  ld_fp_a8(v, src + T.e * 10);
  if (T.active) st_fp_a8(dst + T.e * 10, v.l);
}

// ------------------------------------------------------------------ the pairing check
// f = Miller(G2Base at -sig) (x/crypto optate.go miller with the G2Base lines
// from the table): per doubling f^2 with the line's evaluation at -sig beside
// it (SDBL), then f * line; an addition's line is evaluated beside the
// previous product (LFEVN). Lanes 12..15 evaluate, lanes 0..11 run the Fp12
// job, so the evaluation is free.
//
// The table's lines are normalised (k_g2_lines: c' + b' w + w^3), so f * line
// is 4 products per lane plus the w^3 shift as a linear term.
// (layout S: k_verify_sig's compact team region, see team_final_exp_fc_s)
using ISdbl = XInst<XP_SDBL_S, S_F, S_F>;
using ILfev = XInst<XP_LFEV_S, S_F, S_F>;
using IFeval = XInst<XP_FEVAL_S>;
using ILfix = XInst<XP_LINE_FIX_S, S_F, S_F>;

// The G2Base lines reach the team's registers through one VGPR element per
// lane (lane tl < 4 holds Fp tl of a line: bx.x, bx.y, cy.x, cy.y), read from
// the table one publication ahead, so the L2 latency of the read overlaps the
// rounds between.
struct LinePipe {
  Fp c;
};
HG_DEV void line_fetch(const Team& T, LinePipe& P, const LineCoef* tab, int s) {
  if (T.tl < 4) P.c = reinterpret_cast<const Fp*>(&tab[s])[T.tl];
}
// FBX, FCY of the held line (the evaluation's inputs), then the next line's
// into flight
HG_DEV void publish_line(const Team& T, uint32_t* F, LinePipe& P, const LineCoef* tab, int next) {
  if (T.tl < 4) st_fp(F + (R_FBX_x + T.tl) * 10, P.c);
  team_sync(T);
  if (next < kNumLines) line_fetch(T, P, tab, next);
}

// A signature at infinity contributes e(inf, G2Base) = 1: with SX = NSY = 0
// every evaluated line is w^3, an element of Fp4 the final exponentiation maps
// to 1, so f needs no unit-line substitution.
HG_DEV void team_miller_sig(const Team& T, uint32_t* F, const Fp& sx, const Fp& sy, bool use_s,
                            const LineCoef* tab, XStream& S, XHint after) {
  const int8_t naf[kNafLen] = HG_NAF;
  t12_set_one(T, S_F);
  if (T.tl == 0) {
    Fp zero, one, nsy;
    fp_zero(zero);
    fp_one(one);
    fp_neg(nsy, sy);
    st_fp(F + R_ZERO * 10, zero);
    st_fp(F + R_ONE * 10, one);
    st_fp(F + R_SX * 10, use_s ? sx : zero);
    st_fp(F + R_NSY * 10, use_s ? nsy : zero);
  }
  team_sync(T);
  LinePipe P;
  fp_zero(P.c);
  line_fetch(T, P, tab, 0);
  int s = 0;
  for (int i = kNafLen - 1; i > 0; i--) {
    const int d = naf[i - 1];
    publish_line(T, F, P, tab, s + 1);
    // f^2 (f = 1 on the first digit) beside line s evaluated at -sig
    ISdbl::run(T, S, d != 0 ? xh<ILfev>() : xh<ILfix>());
    const XHint after_digit = i > 1 ? xh<ISdbl>() : xh<IFeval>();
    if (d != 0) {
      publish_line(T, F, P, tab, s + 2);  // read by the evaluation beside f * line s
      ILfev::run(T, S, xh<ILfix>());
      ILfix::run(T, S, after_digit);
      s += 2;
    } else {
      ILfix::run(T, S, after_digit);
      s += 1;
    }
  }
  // the two Frobenius lines
  publish_line(T, F, P, tab, s + 1);
  IFeval::run(T, S, xh<ILfev>());
  publish_line(T, F, P, tab, kNumLines);
  ILfev::run(T, S, xh<ILfix>());
  ILfix::run(T, S, after);
}

// true (team-uniform) when slots a and b hold the same value (both canonical)
HG_DEV bool t12_equal(const Team& T, int a, int b) {
  Fp u, v;
  ld_fp_a8(u, slot(T, a) + T.e * 10);
  ld_fp_a8(v, slot(T, b) + T.e * 10);
  const bool ok = fp_eq(u, v) || !T.active;
  const uint64_t bal = __ballot(ok);
  const int team_shift = (threadIdx.x & 63) & ~15;
  return ((bal >> team_shift) & 0xffffull) == 0xffffull;
}

// FE(Miller(G2Base at -sig)) == Y_r  <=>  e(H, agg) * e(-sig, G2Base) == 1
// kStore: write FE(Miller(G2Base at -sig)) to fe[r] instead (the fold runs
// beside this kernel on a second stream; k_gt_compare finishes the check)
// The team region is layout S (kSigTeamElems, from the generator: slots F..G,
// then the registers from kSigRegBase, the FE pre-pass scratch among them):
// 18.9 KB of LDS per 4-team wave instead of k_verify's 33.9 KB, so the CU's
// LDS holds its four pairing waves and the fold's workgroups beside them, or
// eight pairing waves (two batches in flight) and a fold workgroup.
static constexpr int kSigTeamWords = kSigTeamElems * 10;
static_assert(kSigTeamWords % 2 == 0 && kSigTeamWords <= kTeamWords, "sig team region");
}  // namespace hg
