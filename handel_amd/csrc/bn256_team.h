// bn256_team.h — Fp12 arithmetic spread over a 16-lane "team" (one DPP row).
//
// One pairing check runs on one team. Fp12 = Fp2[w]/(w^6 - xi) is kept flat
// in the team's LDS region as 12 Fp elements: element e = 2k + c holds
// component c (0 = x, the i-coefficient; 1 = y, the real part) of the Fp2
// coefficient of w^k. Lane t < 12 of the team owns element t: for every
// Fp12 product it accumulates its own output coefficient as a sum of
// 26-bit-limb partial products in 64-bit columns and reduces ONCE
// (bn256_fp.h). Lanes 12..15 run the same instruction stream on a clamped
// index and never store, so the wave stays convergent.
//
// The mapping to x/crypto's tower (gfP12{x,y}, gfP6{x,y,z}) is
// c0=y.z, c1=x.z, c2=y.y, c3=x.y, c4=y.x, c5=x.x; values are identical,
// only the storage order differs.
#pragma once
#include "bn256_curve.h"

namespace hg {

static constexpr int kFp12Words = 120;  // 12 elements x 10 limbs

struct Team {
  uint32_t* base;  // this team's LDS slots
  int tl;          // lane within the team, 0..15
  int e;           // owned element, min(tl, 11)
  int k;           // Fp2 coefficient index e >> 1
  int comp;        // 0 = x (imag), 1 = y (real)
  bool active;     // tl < 12
};

HG_DEV uint32_t* slot(const Team& T, int s) { return T.base + s * kFp12Words; }

HG_DEV void ld_fp(Fp& r, const uint32_t* p) {
#pragma unroll
  for (int i = 0; i < 10; i++) r.l[i] = p[i];
}
HG_DEV void st_fp(uint32_t* p, const Fp& a) {
#pragma unroll
  for (int i = 0; i < 10; i++) p[i] = a.l[i];
}
HG_DEV void ld_f2(Fp2& r, const uint32_t* f12, int k) {
  ld_fp(r.x, f12 + (2 * k) * 10);
  ld_fp(r.y, f12 + (2 * k + 1) * 10);
}

HG_DEV void team_sync() { __syncthreads(); }  // blocks are exactly one wave

HG_DEV Team make_team(uint32_t* lds_base, int words_per_team) {
  Team T;
  int team = threadIdx.x >> 4;
  T.tl = threadIdx.x & 15;
  T.base = lds_base + team * words_per_team;
  T.active = T.tl < 12;
  T.e = T.active ? T.tl : 11;
  T.k = T.e >> 1;
  T.comp = T.e & 1;
  return T;
}

// r = T/R mod p for T < 64 p^2 (REDC output < 5p): two conditional subtractions
HG_DEV void acc_reduce_wide(Fp& r, Acc& a) {
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
  // subtract 2p if x >= 2p, then p if x >= p
  const uint32_t p2[10] = {HG_2PLIMBS};
  uint32_t s[10];
  int32_t br = 0;
#pragma unroll
  for (int i = 0; i < 10; i++) {
    int32_t d = (int32_t)x[i] - (int32_t)p2[i] - br;
    br = (d >> 31) & 1;
    s[i] = (uint32_t)d & kMask;
  }
#pragma unroll
  for (int i = 0; i < 10; i++) x[i] = br ? x[i] : s[i];
  fp_csub(r, x);
}

// conditional pieces used by the coefficient kernels
HG_DEV void fp_sel3(Fp& r, int which, const Fp& a, const Fp& b, const Fp& c) {
#pragma unroll
  for (int i = 0; i < 10; i++) r.l[i] = which == 0 ? a.l[i] : (which == 1 ? b.l[i] : c.l[i]);
}

// Given X (Fp2, reduced) and whether the term wraps (multiply by xi), produce
// the two left operands u1, u2 for this lane's component so that
//   comp 0 (x):  out += u1*Y.y + u2*Y.x   with u1 = X'.x, u2 = X'.y
//   comp 1 (y):  out += u1*Y.y + u2*Y.x   with u1 = X'.y, u2 = -X'.x
// where X' = X or xi*X = (3x + y, 3y - x). Operands are loose (< 4p).
HG_DEV void term_operands(Fp& u1, Fp& u2, const Fp2& X, bool wrap, int comp) {
  Fp nx, ny;
  fp_neg_loose(nx, X.x);
  fp_neg_loose(ny, X.y);
  Fp xpx, xpy, nxpx;
#pragma unroll
  for (int i = 0; i < 10; i++) {
    uint32_t x = X.x.l[i], y = X.y.l[i];
    uint32_t wx = 3 * x + y;           // (xi X).x
    uint32_t wy = 3 * y + nx.l[i];     // (xi X).y = 3y - x
    uint32_t wnx = 3 * nx.l[i] + ny.l[i];  // -(xi X).x
    xpx.l[i] = wrap ? wx : x;
    xpy.l[i] = wrap ? wy : y;
    nxpx.l[i] = wrap ? wnx : nx.l[i];
  }
#pragma unroll
  for (int i = 0; i < 10; i++) {
    u1.l[i] = comp ? xpy.l[i] : xpx.l[i];
    u2.l[i] = comp ? nxpx.l[i] : xpy.l[i];
  }
}

// dst = a * b (dst may alias a or b)
HG_DEV void t12_mul(const Team& T, int dst, int sa, int sb) {
  const uint32_t* A = slot(T, sa);
  const uint32_t* B = slot(T, sb);
  Acc acc;
  acc_zero(acc);
#pragma unroll
  for (int i = 0; i < 6; i++) {
    int j = T.k - i;
    bool wrap = j < 0;
    j = wrap ? j + 6 : j;
    Fp2 X, Y;
    ld_f2(X, A, i);
    ld_f2(Y, B, j);
    Fp u1, u2;
    term_operands(u1, u2, X, wrap, T.comp);
    acc_mad(acc, u1, Y.y);
    acc_mad(acc, u2, Y.x);
  }
  Fp r;
  acc_reduce_wide(r, acc);
  team_sync();
  if (T.active) st_fp(slot(T, dst) + T.e * 10, r);
  team_sync();
}

HG_DEV void t12_sqr(const Team& T, int dst, int sa) { t12_mul(T, dst, sa, sa); }

// dst = a * (c + b w + a3 w^3) for line coefficients held in registers
HG_DEV void t12_mul_line(const Team& T, int dst, int sa, const Fp2& la, const Fp2& lb, const Fp2& lc) {
  const uint32_t* A = slot(T, sa);
  Acc acc;
  acc_zero(acc);
  // term j = 0 (c), j = 1 (b), j = 3 (a)
#pragma unroll
  for (int t = 0; t < 3; t++) {
    const int jpos = (t == 0) ? 0 : (t == 1 ? 1 : 3);
    const Fp2& Y = (t == 0) ? lc : (t == 1 ? lb : la);
    int i = T.k - jpos;
    bool wrap = i < 0;
    i = wrap ? i + 6 : i;
    Fp2 X;
    ld_f2(X, A, i);
    Fp u1, u2;
    term_operands(u1, u2, X, wrap, T.comp);
    acc_mad(acc, u1, Y.y);
    acc_mad(acc, u2, Y.x);
  }
  Fp r;
  acc_reduce_wide(r, acc);
  team_sync();
  if (T.active) st_fp(slot(T, dst) + T.e * 10, r);
  team_sync();
}

// dst = conj_p6(a): negate odd powers of w (x/crypto gfP12.Conjugate)
HG_DEV void t12_conj(const Team& T, int dst, int sa) {
  Fp v, n;
  ld_fp(v, slot(T, sa) + T.e * 10);
  fp_neg(n, v);
  fp_sel(v, (T.k & 1) != 0, n, v);
  team_sync();
  if (T.active) st_fp(slot(T, dst) + T.e * 10, v);
  team_sync();
}

__constant__ static const Fp2 kGamma1[6] = HG_GAMMA1;
__constant__ static const Fp kGamma2[6] = HG_GAMMA2;

// dst = a^p (x/crypto gfP12.Frobenius): coefficient k -> conj(a_k) * gamma1[k]
HG_DEV void t12_frob(const Team& T, int dst, int sa) {
  Fp2 X;
  ld_f2(X, slot(T, sa), T.k);
  Fp2 g = kGamma1[T.k];
  // conj(X) = (-x, y); product component comp:
  //   x: (-x) g.y + y g.x ;  y: y g.y + x g.x
  Fp nx;
  fp_neg_loose(nx, X.x);
  Acc acc;
  acc_zero(acc);
  Fp u1, u2;
  fp_sel(u1, T.comp != 0, X.y, nx);
  fp_sel(u2, T.comp != 0, X.x, X.y);
  acc_mad(acc, u1, g.y);
  acc_mad(acc, u2, g.x);
  Fp r;
  acc_reduce(r, acc);
  team_sync();
  if (T.active) st_fp(slot(T, dst) + T.e * 10, r);
  team_sync();
}

// dst = a^(p^2) (gfP12.FrobeniusP2): coefficient k -> a_k * gamma2[k] (gamma2 in Fp)
HG_DEV void t12_frob2(const Team& T, int dst, int sa) {
  Fp v;
  ld_fp(v, slot(T, sa) + T.e * 10);
  Fp g = kGamma2[T.k];
  Fp r;
  fp_mul(r, v, g);
  team_sync();
  if (T.active) st_fp(slot(T, dst) + T.e * 10, r);
  team_sync();
}

HG_DEV void t12_set_one(const Team& T, int dst) {
  Fp v;
  fp_zero(v);
  Fp one;
  fp_one(one);
  fp_sel(v, T.e == 1, one, v);  // element 1 = c0.y
  if (T.active) st_fp(slot(T, dst) + T.e * 10, v);
  team_sync();
}

HG_DEV void t12_copy(const Team& T, int dst, int sa) {
  Fp v;
  ld_fp(v, slot(T, sa) + T.e * 10);
  team_sync();
  if (T.active) st_fp(slot(T, dst) + T.e * 10, v);
  team_sync();
}

// true (team-uniform) when slot s equals 1
HG_DEV bool t12_is_one(const Team& T, int s) {
  Fp v, one, z;
  ld_fp(v, slot(T, s) + T.e * 10);
  fp_one(one);
  fp_zero(z);
  Fp want;
  fp_sel(want, T.e == 1, one, z);
  bool ok = fp_eq(v, want) || !T.active;
  uint64_t bal = __ballot(ok);
  int team_shift = (threadIdx.x & 63) & ~15;
  return ((bal >> team_shift) & 0xffffull) == 0xffffull;
}

// ---------------------------------------------------------------- Fp6 helpers (redundant, per lane)
HG_DEV void f6_inv_lane(Fp2& r0, Fp2& r1, Fp2& r2, const Fp2& c0, const Fp2& c1, const Fp2& c2) {
  Fp2 t0, t1, t2, s, d;
  f2_sqr(t0, c0);
  f2_mul(s, c1, c2);
  f2_mul_xi(s, s);
  f2_sub(t0, t0, s);
  f2_sqr(t1, c2);
  f2_mul_xi(t1, t1);
  f2_mul(s, c0, c1);
  f2_sub(t1, t1, s);
  f2_sqr(t2, c1);
  f2_mul(s, c0, c2);
  f2_sub(t2, t2, s);
  f2_mul(d, c2, t1);
  f2_mul(s, c1, t2);
  f2_add(d, d, s);
  f2_mul_xi(d, d);
  f2_mul(s, c0, t0);
  f2_add(d, d, s);
  f2_inv(d, d);
  f2_mul(r0, t0, d);
  f2_mul(r1, t1, d);
  f2_mul(r2, t2, d);
}

// dst = a^-1 using scratch slots s1, s2 (x/crypto gfP12.Invert)
HG_DEV void t12_inv(const Team& T, int dst, int sa, int s1, int s2) {
  t12_conj(T, s1, sa);          // s1 = conj(a)
  t12_mul(T, s2, sa, s1);       // s2 = a*conj(a) = N (even coefficients only)
  // every lane inverts N (an Fp6 element over tau = w^2) redundantly
  Fp2 n0, n1, n2;
  ld_f2(n0, slot(T, s2), 0);
  ld_f2(n1, slot(T, s2), 2);
  ld_f2(n2, slot(T, s2), 4);
  Fp2 i0, i1, i2;
  f6_inv_lane(i0, i1, i2, n0, n1, n2);
  team_sync();
  {
    // store N^-1 as an Fp12 with zero odd coefficients
    int m = T.k >> 1;
    Fp2 v;
    f2_sel(v, m == 0, i0, (m == 1) ? i1 : i2);
    Fp z, e;
    fp_zero(z);
    e = T.comp ? v.y : v.x;
    fp_sel(e, (T.k & 1) != 0, z, e);
    if (T.active) st_fp(slot(T, s2) + T.e * 10, e);
  }
  team_sync();
  t12_mul(T, dst, s1, s2);  // conj(a) / N
}

// dst = a^u (x/crypto gfP12.Exp with the BN parameter u), dst != sa
HG_DEV void t12_pow_u(const Team& T, int dst, int sa) {
  t12_copy(T, dst, sa);
  for (int bit = 61; bit >= 0; bit--) {
    t12_sqr(T, dst, dst);
    if ((kU >> bit) & 1) t12_mul(T, dst, dst, sa);
  }
}

}  // namespace hg
