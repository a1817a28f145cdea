// bn256_k6.h — Fp12 products of the GT fold on 6-lane teams, Karatsuba in Fp2.
//
// The fold multiplies GT values in HBM into a running product (several waves
// per SIMD: the work is instruction-throughput bound, not latency bound).
// The 12-lane team programs (bn256_xprog.h, MUL12F) give every lane one Fp
// output and compute it as a lazy sum of 12 products: 144 Fp products per
// Fp12 product. Here lane k of a 6-lane team owns the Fp2 coefficient c_k of
// w^k (Fp12 = Fp2[w]/(w^6 - xi), xi = i + 3) and forms
//     c_k = sum_{i+j=k} a_i b_j + sum_{i+j=k+6} (xi a_i) b_j
// with each Fp2 product u v as three Fp products (Karatsuba):
//     t0 = u.y v.y, t1 = u.x v.x, t2 = (u.x + u.y)(v.x + v.y)
//     re = t0 - t1,  im = t2 - t0 - t1
// summed over the six terms as lazy 64-bit column sums T0, T1, T2 and reduced
// twice: 108 Fp products per Fp12 product, and ten teams per wave instead of
// five, so about a fifth fewer lane-instructions per product.
//
// Registers: the fold runs beside the pairing kernel (264 registers a wave),
// so a fold wave must stay within the other 248 of the SIMD's 512. The sums
// run in two passes: T0 and T1 (two accumulators) over the six terms, then
// re = T0 - T1 is reduced and the second accumulator restarts from -(T0 + T1)
// and takes T2. The operand sums u.x + u.y, v.x + v.y are stored beside the
// operands when they are written (slots SA, SX, SB), so pass 2 reads two
// elements per term.
//
// Exactness: every partial product goes into 64-bit columns with no carries.
// im's columns T2 - T0 - T1 are those of sum(u.x v.y + u.y v.x) >= 0, so the
// differences taken mod 2^64 are exact. re's T0 - T1 can be negative per
// column, so T0 starts from kK6C: a multiple of p whose 19 columns are 2^61 +
// (a limb < 2^26) — above any T1 column (60 partial products < 2^54 each).
// Bounds (operands: a canonical, xi a lazy with limbs < 2^28.33, b canonical):
// columns < 2^62.1; re < 2^529.1 and im < 2^516.4 as integers, below p R =
// 2^541.2, so REDC returns < 2p and one conditional subtraction makes every
// output canonical (stored values are compared word for word).
#pragma once
#include "bn256_team.h"

namespace hg {

// 2^61 in columns 0..18, plus the limbs of (-M mod p) in columns 0..9: a
// multiple of p (value ~2^529), generated for this file (see the header note)
static constexpr uint64_t kK6C[19] = {
    0x2000000003e2d72eull, 0x2000000002eac87bull, 0x200000000059ea51ull, 0x20000000032aa9aaull,
    0x200000000019693aull, 0x2000000002fc94a5ull, 0x20000000032fce8eull, 0x20000000030481ceull,
    0x20000000021b99e3ull, 0x200000000016946aull, 0x2000000000000000ull, 0x2000000000000000ull,
    0x2000000000000000ull, 0x2000000000000000ull, 0x2000000000000000ull, 0x2000000000000000ull,
    0x2000000000000000ull, 0x2000000000000000ull, 0x2000000000000000ull};
// (4p)'': 4p with every limb >= 2^26 (top limb 2^23.2), so (4p)'' - x has
// non-negative limbs for canonical x
static constexpr uint32_t kP4L[10] = {0x0422599cu, 0x04ac6c5du, 0x05678616u, 0x05120b5au, 0x07b96e22u,
                                      0x0584dc20u, 0x07fb2e17u, 0x047f9aa5u, 0x078d2a8du, 0x008fb500u};

// Ten 6-lane teams per wave (lanes 6 t .. 6 t + 5; lanes 60..63 idle, team 9's).
static constexpr int kTeams6 = 10;
// Team region: A (12 elements: the running product), B (12: the factor),
// X (12: xi A_k lazily, coefficient 0 unused) — element e = 2k + c at 10 e —
// then the sums x + y of A's, B's and X's six coefficients (6 elements each).
static constexpr int kT6Words = 3 * kFp12Words + 3 * 60;
enum { K6_A = 0, K6_B = 1, K6_X = 2 };
enum { K6_SA = 0, K6_SB = 1, K6_SX = 2 };

struct Team6 {
  uint32_t* base;
  int tl;       // lane within the team, 0..5 (6..9 for lanes 60..63: clamped to 5)
  int k;        // owned Fp2 coefficient
  bool active;  // owns a coefficient (lanes 60..63 do not)
};

HG_DEV int team6_index() {
  const int l = threadIdx.x & 63;
  return l < 60 ? l / 6 : 9;
}
HG_DEV Team6 make_team6(uint32_t* lds_base) {
  Team6 T;
  const int team = team6_index();
  const int l = threadIdx.x & 63;
  T.tl = l - 6 * team;
  T.base = lds_base + team * kT6Words;
  T.active = l < 60;
  T.k = T.active ? T.tl : 5;
  return T;
}
HG_DEV uint32_t* k6_slot(const Team6& T, int s) { return T.base + s * kFp12Words; }
HG_DEV uint32_t* k6_sums(const Team6& T, int s) { return T.base + 3 * kFp12Words + s * 60; }

HG_DEV void acc_init_k6c(Acc& a) {
#pragma unroll
  for (int c = 0; c < 19; c++) a.c[c] = kK6C[c];
  a.c[19] = a.c[20] = 0;
}

// acc += x y, each partial product one v_mad_u64_u32 into its column (the
// empty asm keeps LLVM from re-associating a column into a serial chain)
HG_DEV void acc_mad_pinned6(Acc& a, const Fp& x, const Fp& y) {
#pragma unroll
  for (int i = 0; i < 10; i++)
#pragma unroll
    for (int j = 0; j < 10; j++) {
      a.c[i + j] += (uint64_t)x.l[i] * y.l[j];
      asm("" : "+v"(a.c[i + j]));
    }
}

// pass 1: T0 += u.y v.y, T1 += u.x v.x (two independent chains, interleaved)
HG_DEV void k6_term01(Acc& a0, Acc& a1, const Fp& ux, const Fp& uy, const Fp& vx, const Fp& vy) {
#pragma unroll
  for (int i = 0; i < 10; i++)
#pragma unroll
    for (int j = 0; j < 10; j++) {
      a0.c[i + j] += (uint64_t)uy.l[i] * vy.l[j];
      asm("" : "+v"(a0.c[i + j]));
      a1.c[i + j] += (uint64_t)ux.l[i] * vx.l[j];
      asm("" : "+v"(a1.c[i + j]));
    }
}

// lane k's coefficient of A * B into (cx, cy), canonical; reads A, X, B and
// their sums. Several fold waves share a SIMD, so the operand loads are not
// prefetched (the registers stay free for a wave beside the pairing kernel).
// term i: u = A_i (i <= k) or xi A_i (i > k: wraps past w^6), v = B_(k - i mod 6)
HG_DEV void k6_coeff(const Team6& T, Fp& cx, Fp& cy) {
  Acc a0, a1;
  acc_init_k6c(a0);
  acc_zero(a1);
  const uint32_t* A = k6_slot(T, K6_A);
  const uint32_t* X = k6_slot(T, K6_X);
  const uint32_t* B = k6_slot(T, K6_B);
#pragma unroll
  for (int i = 0; i < 6; i++) {
    const uint32_t* u = (i <= T.k ? A : X) + 20 * i;
    const uint32_t* v = B + 20 * ((T.k - i + 6) % 6);
    Fp ux, uy, vx, vy;
    ld_fp_a8(ux, u);
    ld_fp_a8(uy, u + 10);
    ld_fp_a8(vx, v);
    ld_fp_a8(vy, v + 10);
    k6_term01(a0, a1, ux, uy, vx, vy);
    __builtin_amdgcn_sched_barrier(0);
  }
  // re = T0 + C - T1 (a0 holds T0 + C); a1 restarts at -(T0 + T1) mod 2^64
#pragma unroll
  for (int c = 0; c < 19; c++) {
    const uint64_t t0c = a0.c[c], t1 = a1.c[c];
    a0.c[c] = t0c - t1;
    a1.c[c] = kK6C[c] - t0c - t1;
  }
  acc_reduce(cy, a0);
  // pass 2: im = T2 - T0 - T1, T2 = sum (u.x + u.y)(v.x + v.y)
  const uint32_t* SA = k6_sums(T, K6_SA);
  const uint32_t* SX = k6_sums(T, K6_SX);
  const uint32_t* SB = k6_sums(T, K6_SB);
#pragma unroll
  for (int i = 0; i < 6; i++) {
    Fp su, sv;
    ld_fp_a8(su, (i <= T.k ? SA : SX) + 10 * i);
    ld_fp_a8(sv, SB + 10 * ((T.k - i + 6) % 6));
    acc_mad_pinned6(a1, su, sv);
    __builtin_amdgcn_sched_barrier(0);
  }
  acc_reduce(cx, a1);
}

// lane k stores its coefficient into A and xi times it into X:
// xi (x i + y) = (3x + y) i + (3y - x), the latter as 3y + (4p)'' - x (lazy)
HG_DEV void k6_put(const Team6& T, const Fp& cx, const Fp& cy) {
  if (!T.active) return;
  uint32_t* A = k6_slot(T, K6_A) + 20 * T.k;
  uint32_t* X = k6_slot(T, K6_X) + 20 * T.k;
  uint32_t xx[10], xy[10];
#pragma unroll
  for (int l = 0; l < 10; l++) {
    xx[l] = 3 * cx.l[l] + cy.l[l];
    xy[l] = 3 * cy.l[l] + kP4L[l] - cx.l[l];
  }
  uint32_t sa[10], sx[10];
#pragma unroll
  for (int l = 0; l < 10; l++) {
    sa[l] = cx.l[l] + cy.l[l];
    sx[l] = xx[l] + xy[l];
  }
  st_fp_a8(A, cx.l);
  st_fp_a8(A + 10, cy.l);
  st_fp_a8(X, xx);
  st_fp_a8(X + 10, xy);
  st_fp_a8(k6_sums(T, K6_SA) + 10 * T.k, sa);
  st_fp_a8(k6_sums(T, K6_SX) + 10 * T.k, sx);
}

// A = A * B (then X = xi A): every lane's reads of A and X are done before
// any lane overwrites them
HG_DEV void k6_mul(const Team6& T) {
  team_sync();
  Fp cx, cy;
  k6_coeff(T, cx, cy);
  team_sync();
  k6_put(T, cx, cy);
  team_sync();
}

// ------------------------------------------------------------------ GT values (HBM) <-> 6-lane teams
// lane k moves Fp2 coefficient k (elements 2k, 2k + 1: 20 words)
HG_DEV void k6_read(Fp& x, Fp& y, const Gt* g, const Team6& T) {
  const uint2* src = (const uint2*)__builtin_assume_aligned(g->w + 20 * T.k, 8);
#pragma unroll
  for (int i = 0; i < 5; i++) {
    const uint2 a = src[i], b = src[5 + i];
    x.l[2 * i] = a.x;
    x.l[2 * i + 1] = a.y;
    y.l[2 * i] = b.x;
    y.l[2 * i + 1] = b.y;
  }
}
// the value 1 (coefficient 0 = 1: element 1, the real part)
HG_DEV void k6_one(Fp& x, Fp& y, const Team6& T) {
  fp_zero(x);
  Fp one;
  fp_one(one);
  fp_zero(y);
  fp_sel(y, T.k == 0, one, y);
}
// (x, y) unless keep, else 1: the constants are formed in place, not held
// in registers across a product
HG_DEV void k6_keep_or_one(Fp& x, Fp& y, bool keep, const Team6& T) {
  const bool k0 = T.k == 0;
#pragma unroll
  for (int l = 0; l < 10; l++) {
    x.l[l] = keep ? x.l[l] : 0u;
    y.l[l] = keep ? y.l[l] : (k0 ? onem_limb(l) : 0u);
  }
}
// into slot B; conj: the odd powers of w negated (the inverse of a unitary value)
HG_DEV void k6_put_b(const Team6& T, Fp x, Fp y, bool conj) {
  if (conj && (T.k & 1)) {
    fp_neg(x, x);
    fp_neg(y, y);
  }
  if (!T.active) return;
  uint32_t* B = k6_slot(T, K6_B) + 20 * T.k;
  uint32_t sb[10];
#pragma unroll
  for (int l = 0; l < 10; l++) sb[l] = x.l[l] + y.l[l];
  st_fp_a8(B, x.l);
  st_fp_a8(B + 10, y.l);
  st_fp_a8(k6_sums(T, K6_SB) + 10 * T.k, sb);
}
// into slot A (and X = xi A), for the first factor of a product chain
HG_DEV void k6_put_a(const Team6& T, Fp x, Fp y, bool conj) {
  if (conj && (T.k & 1)) {
    fp_neg(x, x);
    fp_neg(y, y);
  }
  k6_put(T, x, y);
}
HG_DEV void k6_store(const Team6& T, Gt* g) {
  if (!T.active) return;
  Fp x, y;
  const uint32_t* A = k6_slot(T, K6_A) + 20 * T.k;
  ld_fp_a8(x, A);
  ld_fp_a8(y, A + 10);
  uint2* dst = (uint2*)__builtin_assume_aligned(g->w + 20 * T.k, 8);
#pragma unroll
  for (int i = 0; i < 5; i++) {
    dst[i] = make_uint2(x.l[2 * i], x.l[2 * i + 1]);
    dst[5 + i] = make_uint2(y.l[2 * i], y.l[2 * i + 1]);
  }
}

}  // namespace hg
