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
// Fp12 slots of a team's LDS region (tools/gen_g2_schedule.py SLOTS uses the same order)
enum { S_F = 0, S_A, S_B, S_C, S_D, S_E, S_G, S_H, S_I, S_J, S_K, S_L, kSlots };

struct Team {
  uint32_t* base;  // this team's LDS slots
  int tl;          // lane within the team, 0..15
  int e;           // owned element, min(tl, 11)
  int k;           // Fp2 coefficient index e >> 1
  int comp;        // 0 = x (imag), 1 = y (real)
  bool active;     // tl < 12
  // a team spread over the kSplitWaves waves of a workgroup
  // (make_team_split): lane tl of every wave owns element e; a round's
  // products are split between the waves (bn256_xprog.h x_job_split) and
  // team_sync is a workgroup barrier. Only units built with HG_TEAM_SPLIT
  // (below) look at these fields.
  bool split;
  int wave;         // the wave within the workgroup (split teams)
  uint32_t* xchg;   // split teams: this lane's partial-column rows (kXchgWords words per other wave)
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
// 8-byte-aligned element access (every element of a team region: 40-byte
// stride from an 8-aligned base): 64-bit LDS operations, so a 10-limb element
// moves in 3 instructions (2 x ds_read2_b64 + ds_read_b64) instead of 5 x
// ds_read2_b32 — at one wave per SIMD every issued instruction counts.
HG_DEV void ld_fp_a8(Fp& r, const uint32_t* p) {
  const uint64_t* q = (const uint64_t*)__builtin_assume_aligned(p, 8);
#pragma unroll
  for (int i = 0; i < 5; i++) {
    const uint64_t v = q[i];
    r.l[2 * i] = (uint32_t)v;
    r.l[2 * i + 1] = (uint32_t)(v >> 32);
  }
}
HG_DEV void st_fp_a8(uint32_t* p, const uint32_t* l) {
  uint64_t* q = (uint64_t*)__builtin_assume_aligned(p, 8);
#pragma unroll
  for (int i = 0; i < 5; i++) q[i] = (uint64_t)l[2 * i] | ((uint64_t)l[2 * i + 1] << 32);
}
HG_DEV void ld_f2(Fp2& r, const uint32_t* f12, int k) {
  ld_fp(r.x, f12 + (2 * k) * 10);
  ld_fp(r.y, f12 + (2 * k + 1) * 10);
}

// Orders a team's LDS traffic: every lane's earlier LDS writes are seen by
// every lane's later LDS reads. A team lives inside ONE wave, so a wave-level
// barrier is enough (the LDS serves one wave's requests in issue order; the
// wait and the memory clobber keep the compiler from moving LDS accesses
// across it) — and a workgroup barrier would be wrong in k_verify, whose two
// waves run different programs between their shared barriers.
//
// No s_waitcnt: the LDS executes one wave's DS instructions in issue order,
// so a read issued after a write (or a write after a read) of the same wave
// sees it in that order without draining lgkmcnt; the compiler still waits
// for each loaded register before its first use. At one wave per SIMD a
// drain is a parked wave (SQ_WAIT_ANY), never hidden by another wave.
HG_DEV void team_sync() {
#ifdef HG_TEAM_SYNC_DRAIN
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#else
  asm volatile("" ::: "memory");
#endif
  __builtin_amdgcn_wave_barrier();
}

// Split teams exist only in translation units that define HG_TEAM_SPLIT (the
// waves per team) before their includes (bn256_sigw2.hip): everywhere else every branch on Team::split is compiled
// out, so the one-wave kernels' code is untouched.
#ifndef HG_TEAM_SPLIT
#define HG_TEAM_SPLIT 0
#endif
static constexpr bool kTeamSplit = HG_TEAM_SPLIT > 1;
static constexpr int kSplitWaves = HG_TEAM_SPLIT > 1 ? HG_TEAM_SPLIT : 1;

// team_sync for any team: a workgroup barrier when the team spans two waves
HG_DEV void team_sync(const Team& T) {
  if (kTeamSplit && T.split) __syncthreads();
  else team_sync();
}

HG_DEV Team make_team(uint32_t* lds_base, int words_per_team) {
  Team T;
  int team = (threadIdx.x & 63) >> 4;  // teams are numbered within their wave
  T.tl = threadIdx.x & 15;
  T.base = lds_base + team * words_per_team;
  T.active = T.tl < 12;
  T.e = T.active ? T.tl : 11;
  T.k = T.e >> 1;
  T.comp = T.e & 1;
  T.split = false;
  T.wave = 0;
  T.xchg = nullptr;
  return T;
}

// Four 16-lane teams over the kSplitWaves waves of a workgroup: lane tl of
// team t is lane 16 t + tl of EVERY wave; the pairing kernel's latency forms
// (bn256_sigsplit.h). xchg_base: 4 x 16 x (kSplitWaves - 1) x kXchgWords words
// of LDS after the teams' regions (the other waves' partial column sums,
// bn256_xprog.h x_job_split).
static constexpr int kXchgWords = 44;  // 21 64-bit columns, 16-byte aligned rows
HG_DEV Team make_team_split(uint32_t* lds_base, int words_per_team, uint32_t* xchg_base) {
  Team T = make_team(lds_base, words_per_team);
  const int team = (threadIdx.x & 63) >> 4;
  T.split = true;
  T.wave = threadIdx.x >> 6;
  T.xchg = xchg_base + (team * 16 + T.tl) * (kSplitWaves - 1) * kXchgWords;
  return T;
}

// Five 12-lane teams per wave (lanes 12 t .. 12 t + 11; lanes 60..63 are
// team 4's idle lanes 12..15): for programs whose pre-pass values live on
// lanes 0..11 (the generator's PRE_LANES: MUL12F), the GT fold's chunk kernel
// then runs 5 products per wave instruction stream instead of 4.
static constexpr int kTeams12 = 5;
HG_DEV int team12_index() {
  const int l = threadIdx.x & 63;
  return l < 60 ? l / 12 : 4;
}
HG_DEV Team make_team12(uint32_t* lds_base, int words_per_team) {
  Team T;
  const int team = team12_index();
  T.tl = (threadIdx.x & 63) - 12 * team;
  T.base = lds_base + team * words_per_team;
  T.active = T.tl < 12;
  T.e = T.active ? T.tl : 11;
  T.k = T.e >> 1;
  T.comp = T.e & 1;
  T.split = false;
  T.wave = 0;
  T.xchg = nullptr;
  return T;
}

// Reduce a normalized-limb value < 31p (limb 9 holds the top bits) to [0, p):
// q = floor(top / (p9 + 1)) underestimates floor(value / p) by at most one,
// so one conditional subtraction finishes.
HG_DEV void fp_reduce8(Fp& r, const uint32_t* x) {
  constexpr uint32_t p9 = p_top_limb();
  uint32_t q = x[9] / (p9 + 1u);
  uint32_t y[10];
  int32_t c = 0;
#pragma unroll
  for (int i = 0; i < 10; i++) {
    int32_t v = (int32_t)x[i] - (int32_t)(q * p_limb(i)) + c;
    y[i] = (i < 9) ? ((uint32_t)v & kMask) : (uint32_t)v;
    c = v >> 26;
  }
  fp_csub(r, y);  // (the branch-guarded form measured slower here)
}

// REDC of a lazy sum that carries R-shifted linear terms (acc_add_shifted):
// those pass through REDC unchanged, so the result is < (products / R) +
// (linear terms) + p, below 31p (generator-checked); a quotient estimate
// (fp_reduce8) makes it canonical. Sums of products only use acc_reduce.
template <int FROM = 0>
HG_DEV void acc_reduce_wide(Fp& r, Acc& a) {
  acc_redc_digits<FROM>(a);
  uint32_t x[10];
  acc_redc_limbs(x, a);
  fp_reduce8(r, x);
}

// acc_reduce_wide without the final conditional subtraction: the quotient
// estimate leaves the result in [0, 2p) (the lazy rounds, bn256_xprog.h)
template <int FROM = 0>
HG_DEV void acc_reduce_wide_lazy(Fp& r, Acc& a) {
  acc_redc_digits<FROM>(a);
  uint32_t x[10];
  acc_redc_limbs(x, a);
  constexpr uint32_t p9 = p_top_limb();
  const uint32_t q = x[9] / (p9 + 1u);
  int32_t c = 0;
#pragma unroll
  for (int i = 0; i < 10; i++) {
    int32_t v = (int32_t)x[i] - (int32_t)(q * p_limb(i)) + c;
    r.l[i] = (i < 9) ? ((uint32_t)v & kMask) : (uint32_t)v;
    c = v >> 26;
  }
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
  team_sync(T);
  if (T.active) st_fp(slot(T, dst) + T.e * 10, r);
  team_sync(T);
}

HG_DEV void t12_sqr(const Team& T, int dst, int sa) { t12_mul(T, dst, sa, sa); }

// acc += v * R (R = 2^286 = 2^(26*11)): adds the Montgomery-form value v to
// the product sum, i.e. a linear term costs 10 adds instead of a product.
HG_DEV void acc_add_shifted(Acc& acc, const Fp& v) {
#pragma unroll
  for (int i = 0; i < 10; i++) acc.c[kRedcSteps + i] += v.l[i];
}

// small constant multiple of a loose element, limb-wise (no carries)
template <int K>
HG_DEV void fp_scale(Fp& r, const Fp& a) {
#pragma unroll
  for (int i = 0; i < 10; i++) r.l[i] = a.l[i] * K;
}

// dst = a^2 with the symmetric products merged: lane (k, c) sums 4 terms
// (i, j, mult, wrap) over pairs i <= j, i + j = k (mod 6), 8 products.
HG_DEV void t12_sqr_fast(const Team& T, int dst, int sa) {
  const uint32_t* A = slot(T, sa);
  // per-k term tables packed 4 bits per k (k = 0..5): i, j, multiplier, wrap flag
  //   k:      0        1        2        3        4        5
  //   t=0  (1,5,2,w) (0,1,2)  (0,2,2)  (0,3,2)  (0,4,2)  (0,5,2)
  //   t=1  (2,4,2,w) (2,5,2,w)(3,5,2,w)(1,2,2)  (1,3,2)  (1,4,2)
  //   t=2  (0,0,1)   (3,4,2,w)(1,1,1)  (4,5,2,w)(2,2,1)  (2,3,2)
  //   t=3  (3,3,1,w)  -       (4,4,1,w) -       (5,5,1,w) -
  const uint32_t I[4] = {0x000001u, 0x111322u, 0x224130u, 0x050403u};
  const uint32_t J[4] = {0x543215u, 0x432554u, 0x325140u, 0x050403u};
  const uint32_t M[4] = {0x222222u, 0x222222u, 0x212121u, 0x010101u};  // 0 = dummy term
  const uint32_t W[4] = {0x000001u, 0x000111u, 0x001010u, 0x010101u};
  const int sh = 4 * T.k;
  Acc acc;
  acc_zero(acc);
#pragma unroll
  for (int t = 0; t < 4; t++) {
    int i = (I[t] >> sh) & 15, j = (J[t] >> sh) & 15;
    uint32_t m = (M[t] >> sh) & 15;
    bool wrap = ((W[t] >> sh) & 15) != 0;
    Fp2 X, Y;
    ld_f2(X, A, i);
    ld_f2(Y, A, j);
    // the multiplier goes on Y: term_operands negates X, which needs X < p
#pragma unroll
    for (int l = 0; l < 10; l++) {
      Y.x.l[l] *= m;
      Y.y.l[l] *= m;
    }
    Fp u1, u2;
    term_operands(u1, u2, X, wrap, T.comp);
    acc_mad(acc, u1, Y.y);
    acc_mad(acc, u2, Y.x);
  }
  Fp r;
  acc_reduce_wide(r, acc);
  team_sync(T);
  if (T.active) st_fp(slot(T, dst) + T.e * 10, r);
  team_sync(T);
}

// Granger-Scott squaring in the cyclotomic subgroup (valid after the easy part
// of the final exponentiation). With f = (c0 + c3 s) + (c1 + c4 s) w + (c2 + c5 s) w^2,
// s = w^3, each group (a, b) squares in Fp4: (a^2 + xi b^2) + 2ab s, and
//   c0' = 3(a^2 + xi b^2) - 2c0   c3' = 6ab + 2c3      for (a, b) = (c0, c3)
//   c2' = 3(a^2 + xi b^2) - 2c2   c5' = 6ab + 2c5      for (a, b) = (c1, c4)
//   c4' = 3(a^2 + xi b^2) - 2c4   c1' = 6 xi ab + 2c1  for (a, b) = (c2, c5)
// Each lane: 3 products; the +-2c term is added to the high columns.
HG_DEV void t12_cyc_sqr(const Team& T, int dst, int sa) {
  const uint32_t* A = slot(T, sa);
  const int k = T.k;
  const int ga = (k == 0 || k == 3) ? 0 : ((k == 2 || k == 5) ? 1 : 2);
  const bool sq = (k & 1) == 0;   // k = 0, 2, 4: the a^2 + xi b^2 lanes
  const bool xi = (k == 1);       // the 6 xi ab lane
  const bool cx = T.comp == 0;
  Fp2 a, b;
  ld_f2(a, A, ga);
  ld_f2(b, A, ga + 3);
  Fp c;
  ld_fp(c, A + T.e * 10);
  Fp nax, nay, nbx, da, db, sa_, sb_;
  fp_neg_loose(nax, a.x);
  fp_neg_loose(nay, a.y);
  fp_neg_loose(nbx, b.x);
  fp_sub(da, a.y, a.x);
  fp_sub(db, b.y, b.x);
  fp_add_loose(sa_, a.y, a.x);
  fp_add_loose(sb_, b.y, b.x);
  Fp u1, v1, u2, v2, u3;
#pragma unroll
  for (int l = 0; l < 10; l++) {
    // sq lanes: x: (6ax)ay + (18bx)by + (3sb)db ; y: (3sa)da + (6nbx)by + (9sb)db
    // ab lanes: x: (6ax)by + (6ay)bx ; y: (6ay)by + (6nax)bx
    // xi lane:  x: 6(3ax+ay)by + 6(3ay+nax)bx ; y: 6(3ay+nax)by + 6(3nax+nay)bx
    uint32_t xa = 3 * a.x.l[l] + a.y.l[l], xb = 3 * a.y.l[l] + nax.l[l], xc = 3 * nax.l[l] + nay.l[l];
    uint32_t sq_u1 = cx ? 6 * a.x.l[l] : 3 * sa_.l[l];
    uint32_t sq_v1 = cx ? a.y.l[l] : da.l[l];
    uint32_t sq_u2 = cx ? 18 * b.x.l[l] : 6 * nbx.l[l];
    uint32_t ab_u1 = xi ? 6 * (cx ? xa : xb) : 6 * (cx ? a.x.l[l] : a.y.l[l]);
    uint32_t ab_u2 = xi ? 6 * (cx ? xb : xc) : 6 * (cx ? a.y.l[l] : nax.l[l]);
    u1.l[l] = sq ? sq_u1 : ab_u1;
    v1.l[l] = sq ? sq_v1 : b.y.l[l];
    u2.l[l] = sq ? sq_u2 : ab_u2;
    v2.l[l] = sq ? b.y.l[l] : b.x.l[l];
    u3.l[l] = sq ? (cx ? 3 * sb_.l[l] : 9 * sb_.l[l]) : 0u;
  }
  Acc acc;
  acc_zero(acc);
  acc_mad(acc, u1, v1);
  acc_mad(acc, u2, v2);
  acc_mad(acc, u3, db);
  // linear term: -2c on the a^2 lanes, +2c on the others (added as 2c R or 2(p - c) R)
  Fp nc, lin;
  fp_neg_loose(nc, c);
  fp_sel(lin, sq, nc, c);
  fp_scale<2>(lin, lin);
  acc_add_shifted(acc, lin);
  Fp r;
  acc_reduce_wide(r, acc);
  team_sync(T);
  if (T.active) st_fp(slot(T, dst) + T.e * 10, r);
  team_sync(T);
}

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
  team_sync(T);
  if (T.active) st_fp(slot(T, dst) + T.e * 10, r);
  team_sync(T);
}

// dst = conj_p6(a): negate odd powers of w (x/crypto gfP12.Conjugate)
HG_DEV void t12_conj(const Team& T, int dst, int sa) {
  Fp v, n;
  ld_fp(v, slot(T, sa) + T.e * 10);
  fp_neg(n, v);
  fp_sel(v, (T.k & 1) != 0, n, v);
  team_sync(T);
  if (T.active) st_fp(slot(T, dst) + T.e * 10, v);
  team_sync(T);
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
  team_sync(T);
  if (T.active) st_fp(slot(T, dst) + T.e * 10, r);
  team_sync(T);
}

// dst = a^(p^2) (gfP12.FrobeniusP2): coefficient k -> a_k * gamma2[k] (gamma2 in Fp)
HG_DEV void t12_frob2(const Team& T, int dst, int sa) {
  Fp v;
  ld_fp(v, slot(T, sa) + T.e * 10);
  Fp g = kGamma2[T.k];
  Fp r;
  fp_mul(r, v, g);
  team_sync(T);
  if (T.active) st_fp(slot(T, dst) + T.e * 10, r);
  team_sync(T);
}

HG_DEV void t12_set_one(const Team& T, int dst) {
  Fp v;
  fp_zero(v);
  Fp one;
  fp_one(one);
  fp_sel(v, T.e == 1, one, v);  // element 1 = c0.y
  if (T.active) st_fp(slot(T, dst) + T.e * 10, v);
  team_sync(T);
}

HG_DEV void t12_copy(const Team& T, int dst, int sa) {
  Fp v;
  ld_fp(v, slot(T, sa) + T.e * 10);
  team_sync(T);
  if (T.active) st_fp(slot(T, dst) + T.e * 10, v);
  team_sync(T);
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

// slot s2 holds N = a conj(a) (an Fp6 element over tau = w^2: odd coefficients
// zero); replaces it by N^-1 = adj(N) / d (x/crypto gfP6.Invert:
// t0 = c0^2 - xi c1 c2, t1 = xi c2^2 - c0 c1, t2 = c1^2 - c0 c2,
// d = xi (c2 t1 + c1 t2) + c0 t0). The adjugate's three products and d's
// three terms are split over lanes 0..2 with one instruction stream (lane j
// computes term j; the odd, zero coefficients of s2 carry them between lanes),
// so a lane runs 2 + 1 Fp2 products instead of 9; the Fp2 inversion of d (one
// Bernstein-Yang Fp inversion) runs on every lane, and each lane finishes
// its own element of N^-1 with one lazy sum of two products.
HG_DEV void t12_inv_norm(const Team& T, int s2) {
  uint32_t* N = slot(T, s2);
  Fp2 c0, c1, c2;
  ld_f2(c0, N, 0);
  ld_f2(c1, N, 2);
  ld_f2(c2, N, 4);
  const int j = T.tl < 3 ? T.tl : 2;
  // t_j = alpha X^2 - beta Y Z with (X, alpha; Y, Z, beta) per j
  Fp2 X, Y, Z, u, v, t;
  f2_sel(X, j == 0, c0, j == 1 ? c2 : c1);
  f2_sel(Y, j == 0, c1, c0);
  f2_sel(Z, j == 1, c1, c2);
  f2_sqr(u, X);
  f2_mul(v, Y, Z);
  Fp2 xu, xv;
  f2_mul_xi(xu, u);
  f2_mul_xi(xv, v);
  f2_sel(u, j == 1, xu, u);
  f2_sel(v, j == 0, xv, v);
  f2_sub(t, u, v);
  team_sync(T);
  if (T.tl < 3) {  // odd coefficient 2j + 1 of s2
    st_fp(N + (4 * j + 2) * 10, t.x);
    st_fp(N + (4 * j + 3) * 10, t.y);
  }
  team_sync(T);
  Fp2 t0, t1, t2;
  ld_f2(t0, N, 1);
  ld_f2(t1, N, 3);
  ld_f2(t2, N, 5);
  // term j of d: c2 t1, c1 t2, c0 t0
  Fp2 P, Q, w;
  f2_sel(P, j == 0, c2, j == 1 ? c1 : c0);
  f2_sel(Q, j == 0, t1, j == 1 ? t2 : t0);
  f2_mul(w, P, Q);
  team_sync(T);
  if (T.tl < 3) {
    st_fp(N + (4 * j + 2) * 10, w.x);
    st_fp(N + (4 * j + 3) * 10, w.y);
  }
  team_sync(T);
  Fp2 w0, w1, w2, d;
  ld_f2(w0, N, 1);
  ld_f2(w1, N, 3);
  ld_f2(w2, N, 5);
  f2_add(d, w0, w1);
  f2_mul_xi(d, d);
  f2_add(d, d, w2);
#ifndef HG_PROBE_NOINV  // timing probe only (wrong values): the inversion's share of a pairing kernel
  f2_inv(d, d);
#endif
  // element e of N^-1: component comp of t_m d^-1 (m = k / 2), zero for odd k
  const int m = T.k >> 1;
  Fp2 tm;
  f2_sel(tm, m == 0, t0, m == 1 ? t1 : t2);
  // x (imag) = tm.x d.y + tm.y d.x; y (real) = tm.y d.y - tm.x d.x
  Fp a1, b1, ntx;
  fp_neg_loose(ntx, tm.x);
  fp_sel(a1, T.comp != 0, tm.y, tm.x);
  fp_sel(b1, T.comp != 0, ntx, tm.y);
  Acc acc;
  acc_zero(acc);
  acc_mad(acc, a1, d.y);
  acc_mad(acc, b1, d.x);
  Fp e, z;
  acc_reduce(e, acc);
  fp_zero(z);
  fp_sel(e, (T.k & 1) != 0, z, e);
  team_sync(T);
  if (T.active) st_fp(N + T.e * 10, e);
  team_sync(T);
}

// t12_inv_norm in two halves around its one Fp inversion, for kernels that
// invert the norms of a whole batch of checks at once (bn256_sig12.hip: one
// batched inversion per 256 checks instead of one Bernstein-Yang inversion
// per wave, 4.3 % of the 12-lane pairing kernel's VALU instructions,
// profiles/r06p_inv_probe.json). _terms runs t12_inv_norm up to d (the
// adjugate's terms t0, t1, t2 and d, team-uniform, every lane holds them) and
// returns n = |d|^2 as f2_inv forms it; _finish, given n^-1, writes N^-1
// into slot s2 exactly as t12_inv_norm does (the same products in the same
// order: identical canonical values).
struct NormTerms {
  Fp2 t0, t1, t2, d;
};
HG_DEV void t12_inv_norm_terms(const Team& T, int s2, NormTerms& o, Fp& nrm) {
  uint32_t* N = slot(T, s2);
  Fp2 c0, c1, c2;
  ld_f2(c0, N, 0);
  ld_f2(c1, N, 2);
  ld_f2(c2, N, 4);
  const int j = T.tl < 3 ? T.tl : 2;
  Fp2 X, Y, Z, u, v, t;
  f2_sel(X, j == 0, c0, j == 1 ? c2 : c1);
  f2_sel(Y, j == 0, c1, c0);
  f2_sel(Z, j == 1, c1, c2);
  f2_sqr(u, X);
  f2_mul(v, Y, Z);
  Fp2 xu, xv;
  f2_mul_xi(xu, u);
  f2_mul_xi(xv, v);
  f2_sel(u, j == 1, xu, u);
  f2_sel(v, j == 0, xv, v);
  f2_sub(t, u, v);
  team_sync(T);
  if (T.tl < 3) {
    st_fp(N + (4 * j + 2) * 10, t.x);
    st_fp(N + (4 * j + 3) * 10, t.y);
  }
  team_sync(T);
  ld_f2(o.t0, N, 1);
  ld_f2(o.t1, N, 3);
  ld_f2(o.t2, N, 5);
  Fp2 P, Q, w;
  f2_sel(P, j == 0, c2, j == 1 ? c1 : c0);
  f2_sel(Q, j == 0, o.t1, j == 1 ? o.t2 : o.t0);
  f2_mul(w, P, Q);
  team_sync(T);
  if (T.tl < 3) {
    st_fp(N + (4 * j + 2) * 10, w.x);
    st_fp(N + (4 * j + 3) * 10, w.y);
  }
  team_sync(T);
  Fp2 w0, w1, w2;
  ld_f2(w0, N, 1);
  ld_f2(w1, N, 3);
  ld_f2(w2, N, 5);
  f2_add(o.d, w0, w1);
  f2_mul_xi(o.d, o.d);
  f2_add(o.d, o.d, w2);
  Acc acc;  // f2_inv's norm
  acc_zero(acc);
  acc_sqr(acc, o.d.x);
  acc_sqr(acc, o.d.y);
  acc_reduce(nrm, acc);
}
HG_DEV void t12_inv_norm_finish(const Team& T, int s2, const NormTerms& o, const Fp& ninv) {
  uint32_t* N = slot(T, s2);
  Fp2 d;  // d^-1, as f2_inv
  Fp ndx;
  fp_neg(ndx, o.d.x);
  fp_mul(d.x, ndx, ninv);
  fp_mul(d.y, o.d.y, ninv);
  const int m = T.k >> 1;
  Fp2 tm;  // (selects on values: a select between member references spills to scratch)
  f2_sel(tm, m == 1, o.t1, o.t2);
  f2_sel(tm, m == 0, o.t0, tm);
  Fp a1, b1, ntx;
  fp_neg_loose(ntx, tm.x);
  fp_sel(a1, T.comp != 0, tm.y, tm.x);
  fp_sel(b1, T.comp != 0, ntx, tm.y);
  Acc acc;
  acc_zero(acc);
  acc_mad(acc, a1, d.y);
  acc_mad(acc, b1, d.x);
  Fp e, z;
  acc_reduce(e, acc);
  fp_zero(z);
  fp_sel(e, (T.k & 1) != 0, z, e);
  team_sync(T);
  if (T.active) st_fp(N + T.e * 10, e);
  team_sync(T);
}

// dst = a^-1 using scratch slots s1, s2 (x/crypto gfP12.Invert)
HG_DEV void t12_inv(const Team& T, int dst, int sa, int s1, int s2) {
  t12_conj(T, s1, sa);          // s1 = conj(a)
  t12_mul(T, s2, sa, s1);       // s2 = a*conj(a) = N (even coefficients only)
  t12_inv_norm(T, s2);
  t12_mul(T, dst, s1, s2);      // conj(a) / N
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
