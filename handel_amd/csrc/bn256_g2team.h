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

// Montgomery REDC of a lazy sum (T < p R), canonical result.
HG_DEV void acc_reduce8(Fp& r, Acc& a) { acc_reduce_wide(r, a); }

// sum_m c_m * F[r_m] + K p  (K = sum of the negative |c_m|): a non-negative
// value < (sum |c_m|) p with normalized limbs. Coefficients are small
// (|sum| <= 24, checked by the generator), so limb sums fit in int32.
// Operand address: F register (< 128), element of Fp12 slot A (128..139) or B (160..171).
HG_DEV const uint32_t* op_addr(const uint32_t* F, const uint32_t* A, const uint32_t* B, uint32_t r) {
  const uint32_t* base = (r & 128u) ? ((r & 32u) ? B : A) : F;
  return base + (r & 31u) * 10 + ((r & 128u) ? 0u : (r & 96u) * 10);
}

HG_DEV void g2_lincomb(Fp& out, const uint32_t* F, const uint32_t* A, const uint32_t* B, const uint8_t* rr,
                       const int8_t* cc, int nt) {
  int32_t v[10];
#pragma unroll
  for (int i = 0; i < 10; i++) v[i] = 0;
  int32_t negk = 0;
  for (int m = 0; m < nt; m++) {
    const uint32_t* x = op_addr(F, A, B, rr[m]);
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

// One round: every lane computes its dst = sum_slot lincomb_a * lincomb_b.
// A, B: Fp12 source slots; D: Fp12 destination slot (dst codes >= 128).
HG_DEV void g2_round(const Team& T, uint32_t* F, const uint32_t* A, const uint32_t* B, uint32_t* D,
                     const G2Round& R) {
  const G2Lane& L = kG2Lanes[R.first + T.tl];
  Acc acc;
  acc_zero(acc);
#pragma unroll
  for (int s = 0; s < kG2MaxSlots; s++) {
    if (s < R.nslot) {
      Fp a, b;
      g2_lincomb(a, F, A, B, L.ar[s], L.ac[s], R.nta[s]);
      g2_lincomb(b, F, A, B, L.br[s], L.bc[s], R.ntb[s]);
      acc_mad(acc, a, b);
    }
  }
  Fp r;
  acc_reduce8(r, acc);
  uint32_t dst = L.dst;
  team_sync();
  if (dst != kG2None) st_fp(((dst & 128u) ? D + (dst & 31u) * 10 : F + dst * 10), r);
  team_sync();
}

template <int N>
HG_DEV void g2_program(const Team& T, uint32_t* F, const G2Round (&prog)[N]) {
#pragma unroll
  for (int i = 0; i < N; i++) g2_round(T, F, F, F, F, prog[i]);
}

// The same Fp12 squarings as table programs (kProgSQR12 / kProgCYC_SQR); the
// specialised index-arithmetic versions in bn256_team.h are what the kernels
// run, these stay as a cross-check of the generated tables.
HG_DEV void t12_sqr_table(const Team& T, uint32_t* F, int dst, int sa) {
  g2_round(T, F, slot(T, sa), slot(T, sa), slot(T, dst), kProgSQR12[0]);
}
HG_DEV void t12_cyc_sqr_table(const Team& T, uint32_t* F, int dst, int sa) {
  g2_round(T, F, slot(T, sa), slot(T, sa), slot(T, dst), kProgCYC_SQR[0]);
}
HG_DEV void t12_sqr_fast(const Team& T, uint32_t* F, int dst, int sa) { t12_sqr_fast(T, dst, sa); }
HG_DEV void t12_cyc_sqr(const Team& T, uint32_t* F, int dst, int sa) { t12_cyc_sqr(T, dst, sa); }
__constant__ static const int8_t kUNaf3[kUNaf3Len] = HG_U_NAF3;

// dst = a^u (x/crypto gfP12.Exp(t, u)) for a in the cyclotomic subgroup, where
// a^-1 = conj(a): width-3 signed digits of u, so the multipliers are a, a^3
// and their conjugates (62 cyclotomic squarings + 16 multiplications instead
// of 62 + 29 for the binary expansion). s3, si, s3i: scratch slots; dst and
// the scratch slots must differ from sa.
HG_DEV void t12_pow_u_cyc(const Team& T, uint32_t* F, int dst, int sa, int s3, int si, int s3i) {
  t12_cyc_sqr(T, s3, sa);
  t12_mul(T, s3, s3, sa);   // a^3
  t12_conj(T, si, sa);      // a^-1
  t12_conj(T, s3i, s3);     // a^-3
  static_assert(HG_U_NAF3_TOP == 3, "top digit of the width-3 NAF of u");
  t12_copy(T, dst, s3);
  for (int i = kUNaf3Len - 2; i >= 0; i--) {
    t12_cyc_sqr(T, dst, dst);
    const int d = kUNaf3[i];
    if (d != 0) t12_mul(T, dst, dst, d == 1 ? sa : (d == 3 ? s3 : (d == -1 ? si : s3i)));
  }
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
