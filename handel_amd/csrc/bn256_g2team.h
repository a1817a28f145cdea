// bn256_g2team.h — executes the generated lane-parallel G2 schedule
// (bn256_g2sched.h, from tools/gen_g2_schedule.py) on a 16-lane team.
//
// The team keeps an LDS "register file" F of Fp elements (the Miller-loop
// point R = (X, Y, Z, T), the pk Q and its Frobenius images, the G1 points,
// line coefficients and temporaries). A round makes every lane compute
//   dst = sum_slot lincomb_a * lincomb_b
// with one lazy Montgomery reduction; lanes differ only in the LDS addresses
// and small coefficients they read from the schedule table. This replaces
// the per-lane redundant evaluation of lineFunctionDouble / lineFunctionAdd
// (x/crypto optate.go) by a 3-round (double) / 5-round (add) team program.
#pragma once
#include "bn256_g2sched.h"
#include "bn256_team.h"

namespace hg {

// Reduce a normalized-limb value < 8p (limb 9 holds the top bits) to [0, p).
HG_DEV void fp_reduce8(Fp& r, const uint32_t* x) {
  constexpr uint32_t p9 = p_top_limb();
  uint32_t q = x[9] / (p9 + 1u);  // floor(value/p) - {0, 1}
  uint32_t y[10];
  int32_t c = 0;
#pragma unroll
  for (int i = 0; i < 10; i++) {
    int32_t v = (int32_t)x[i] - (int32_t)(q * p_limb(i)) + c;
    y[i] = (i < 9) ? ((uint32_t)v & kMask) : (uint32_t)v;
    c = v >> 26;
  }
  fp_csub(r, y);
}

// Montgomery REDC for T < ~199 p^2 (output < 8p), then full reduction.
HG_DEV void acc_reduce8(Fp& r, Acc& a) {
#pragma unroll
  for (int i = 0; i < 10; i++) {
    uint32_t q = ((uint32_t)a.c[i] * kPInv26) & kMask;
#pragma unroll
    for (int j = 0; j < 10; j++) a.c[i + j] += (uint64_t)q * p_limb(j);
    a.c[i + 1] += a.c[i] >> 26;
  }
  uint32_t x[10];
  uint64_t carry = 0;
#pragma unroll
  for (int j = 0; j < 10; j++) {
    uint64_t v = a.c[10 + j] + carry;
    x[j] = (j < 9) ? ((uint32_t)v & kMask) : (uint32_t)v;
    carry = v >> 26;
  }
  fp_reduce8(r, x);
}

// sum_m c_m * F[r_m] + K p  (K = sum of the negative |c_m|): a non-negative
// value < (sum |c_m|) p with normalized limbs. Coefficients are small
// (|sum| <= 24, checked by the generator), so limb sums fit in int32.
HG_DEV void g2_lincomb(Fp& out, const uint32_t* F, const uint8_t* rr, const int8_t* cc, int nt) {
  int32_t v[10];
#pragma unroll
  for (int i = 0; i < 10; i++) v[i] = 0;
  int32_t negk = 0;
  for (int m = 0; m < nt; m++) {
    const uint32_t* x = F + rr[m] * 10;
    int32_t k = cc[m];
    negk += k < 0 ? -k : 0;
#pragma unroll
    for (int i = 0; i < 10; i++) v[i] += k * (int32_t)x[i];
  }
  int32_t c = 0;
#pragma unroll
  for (int i = 0; i < 10; i++) {
    int32_t t = v[i] + negk * (int32_t)p_limb(i) + c;
    out.l[i] = (i < 9) ? ((uint32_t)t & kMask) : (uint32_t)t;
    c = t >> 26;
  }
}

HG_DEV void g2_round(const Team& T, uint32_t* F, const G2Round& R) {
  const G2Lane& L = kG2Lanes[R.first + T.tl];
  Acc acc;
  acc_zero(acc);
#pragma unroll
  for (int s = 0; s < 3; s++) {
    if (s < R.nslot) {
      Fp a, b;
      g2_lincomb(a, F, L.ar[s], L.ac[s], R.nta[s]);
      g2_lincomb(b, F, L.br[s], L.bc[s], R.ntb[s]);
      acc_mad(acc, a, b);
    }
  }
  Fp r;
  acc_reduce8(r, acc);
  uint8_t dst = L.dst;
  team_sync();
  if (dst != kG2None) st_fp(F + dst * 10, r);
  team_sync();
}

template <int N>
HG_DEV void g2_program(const Team& T, uint32_t* F, const G2Round (&prog)[N]) {
#pragma unroll
  for (int i = 0; i < N; i++) g2_round(T, F, prog[i]);
}

// dst = a * (c + b w + a3 w^3) with the line coefficients in the register
// file: ra, rb, rc are the x-component register indices of the Fp2 regs.
HG_DEV void t12_mul_line_regs(const Team& T, int dst, int sa, const uint32_t* F, int ra, int rb, int rc) {
  Fp2 la, lb, lc;
  ld_fp(la.x, F + ra * 10);
  ld_fp(la.y, F + (ra + 1) * 10);
  ld_fp(lb.x, F + rb * 10);
  ld_fp(lb.y, F + (rb + 1) * 10);
  ld_fp(lc.x, F + rc * 10);
  ld_fp(lc.y, F + (rc + 1) * 10);
  t12_mul_line(T, dst, sa, la, lb, lc);
}

}  // namespace hg
