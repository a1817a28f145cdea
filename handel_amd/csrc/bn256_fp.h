// bn256_fp.h — 256-bit prime-field arithmetic for the dclxvi BN256 curve on
// gfx950 (CDNA4).
//
// The curve is the one golang.org/x/crypto/bn256 and cloudflare/bn256
// implement (bn256/go/bn256.go:17, bn256/cf/bn256.go:17):
//   p = 36u^4 + 36u^3 + 24u^2 + 6u + 1, u = 6518589491078791937 (p > 2^255).
//
// Representation (chosen for v_mad_u64_u32, which is half-rate on gfx950):
//   * an element is 10 limbs of 26 bits (little-endian), Montgomery form with
//     R = 2^286 (11 REDC digits), fully reduced to [0, p) unless a function
//     says otherwise;
//   * a product is accumulated column-wise into 21 x 64-bit accumulators
//     (`Acc`). Each 26x26-bit partial product is ONE in-place
//     v_mad_u64_u32 with no carry handling, and a column has room for 2^12
//     partial products, so a sum of up to 16 products of reduced operands
//     is reduced ONCE (lazy reduction) — the Fp12 coefficient sums, the Fp2
//     schoolbook products and the squarings all use that.
//   * Montgomery REDC of T < p R (R = 2^286 ~ 2^30.5 p, so any lazy sum the
//     code forms) returns a value < 2p, and one conditional subtraction makes
//     it canonical. The 11th digit costs 10 mads and saves a quotient-estimate
//     reduction after every lazy sum.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bn256_constants.h"
#include "bn256_inv.h"

#define HG_DEV __device__ __forceinline__

namespace hg {

struct Fp {
  uint32_t l[10];
};
struct Acc {
  uint64_t c[21];  // product columns 0..18, REDC digits up to 19, R-shifted terms 11..20
};

static constexpr uint32_t kPLimbsC[10] = {HG_PLIMBS};
__host__ __device__ constexpr uint32_t p_top_limb() { return kPLimbsC[9]; }

HG_DEV uint32_t p_limb(int i) {
  // folded to an immediate after unrolling
  const uint32_t pl[10] = {HG_PLIMBS};
  return pl[i];
}
HG_DEV uint32_t onem_limb(int i) {
  const uint32_t o[10] = {HG_ONE_M};
  return o[i];
}

HG_DEV void fp_zero(Fp& r) {
#pragma unroll
  for (int i = 0; i < 10; i++) r.l[i] = 0;
}
HG_DEV void fp_one(Fp& r) {
#pragma unroll
  for (int i = 0; i < 10; i++) r.l[i] = onem_limb(i);
}
HG_DEV bool fp_is_zero(const Fp& a) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 10; i++) o |= a.l[i];
  return o == 0;
}
HG_DEV bool fp_eq(const Fp& a, const Fp& b) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 10; i++) o |= a.l[i] ^ b.l[i];
  return o == 0;
}
HG_DEV void fp_sel(Fp& r, bool c, const Fp& a, const Fp& b) {
#pragma unroll
  for (int i = 0; i < 10; i++) r.l[i] = c ? a.l[i] : b.l[i];
}

// r = x - p if x >= p else x, for normalized x < 2p (limb 9 may hold up to 27 bits)
HG_DEV void fp_csub(Fp& r, const uint32_t* x) {
  uint32_t s[10];
  int32_t br = 0;
#pragma unroll
  for (int i = 0; i < 10; i++) {
    int32_t t = (int32_t)x[i] - (int32_t)p_limb(i) - br;
    br = (t >> 31) & 1;
    s[i] = (uint32_t)t & kMask;
  }
  bool keep = br != 0;  // borrow out => x < p
#pragma unroll
  for (int i = 0; i < 10; i++) r.l[i] = keep ? x[i] : s[i];
}

// fp_csub for REDC outputs: x >= p implies x9 >= p9, and a REDC output of a
// lazy sum is below p + T/R with T/R far below 2^234, so x9 >= p9 happens for
// about one lane in 2^22. The subtraction runs under that (exact) test, so the
// wave normally skips it with one compare and a branch instead of a 10-limb
// borrow chain and 10 selects — at one wave per SIMD every instruction counts.
HG_DEV void fp_csub_rare(Fp& r, const uint32_t* x) {
  uint32_t v[10];
#pragma unroll
  for (int i = 0; i < 10; i++) v[i] = x[i];
  if (__builtin_expect(x[9] >= p_top_limb(), 0)) {
    uint32_t s[10];
    int32_t br = 0;
#pragma unroll
    for (int i = 0; i < 10; i++) {
      int32_t t = (int32_t)x[i] - (int32_t)p_limb(i) - br;
      br = (t >> 31) & 1;
      s[i] = (uint32_t)t & kMask;
    }
    if (br == 0) {
#pragma unroll
      for (int i = 0; i < 10; i++) v[i] = s[i];
    }
  }
#pragma unroll
  for (int i = 0; i < 10; i++) r.l[i] = v[i];
}

// ---------------------------------------------------------------- accumulators
HG_DEV void acc_zero(Acc& a) {
#pragma unroll
  for (int i = 0; i < 21; i++) a.c[i] = 0;
}
// a += x * y (limbs of x, y may be up to 27 bits: sums of two reduced values)
HG_DEV void acc_mad(Acc& a, const Fp& x, const Fp& y) {
#pragma unroll
  for (int i = 0; i < 10; i++)
#pragma unroll
    for (int j = 0; j < 10; j++) a.c[i + j] += (uint64_t)x.l[i] * y.l[j];
}
// a += x^2 (55 partial products)
HG_DEV void acc_sqr(Acc& a, const Fp& x) {
  uint32_t d[10];
#pragma unroll
  for (int i = 0; i < 10; i++) d[i] = x.l[i] << 1;
#pragma unroll
  for (int i = 0; i < 10; i++) {
    a.c[2 * i] += (uint64_t)x.l[i] * x.l[i];
#pragma unroll
    for (int j = i + 1; j < 10; j++) a.c[i + j] += (uint64_t)x.l[i] * d[j];
  }
}
// One Montgomery REDC digit: q = c_i p' mod 2^26, c += q p 2^(26 i), and the
// (now zero mod 2^26) column i carries into column i + 1.
HG_DEV void acc_redc_digit(Acc& a, int i) {
  const uint32_t q = ((uint32_t)a.c[i] * kPInv26) & kMask;
#pragma unroll
  for (int j = 0; j < 10; j++) {
    a.c[i + j] += (uint64_t)q * p_limb(j);
    asm("" : "+v"(a.c[i + j]));  // no reassociation into per-column chains
  }
  a.c[i + 1] += a.c[i] >> 26;
}
// digits FROM .. 10 (FROM > 0: acc_mad_redc ran the first ones)
template <int FROM>
HG_DEV void acc_redc_digits(Acc& a) {
#pragma unroll
  for (int i = FROM; i < kRedcSteps; i++) acc_redc_digit(a, i);
}
// columns 11..20 of a reduced accumulator as 10 limbs (the top one unmasked)
HG_DEV void acc_redc_limbs(uint32_t (&x)[10], const Acc& a) {
  uint64_t carry = 0;
#pragma unroll
  for (int j = 0; j < 10; j++) {
    uint64_t v = a.c[kRedcSteps + j] + carry;
    x[j] = (j < 9) ? ((uint32_t)v & kMask) : (uint32_t)v;
    carry = v >> 26;
  }
}
// a += x * y with the REDC digits interleaved, for the LAST product of a lazy
// sum: once row i of x * y is in, column i is complete (earlier products are
// whole, rows > i only reach higher columns), so digit i runs right there.
// The reduction's serial chain (column i -> q_i -> 10 mads -> carry into
// column i + 1) then overlaps the next rows' independent mads instead of
// trailing all the products, where one wave per SIMD has nothing to hide it
// behind. Digits 0..9; digit 10 follows (acc_reduce<10> and its wide forms).
HG_DEV void acc_mad_redc(Acc& a, const Fp& x, const Fp& y) {
#pragma unroll
  for (int i = 0; i < 10; i++) {
#pragma unroll
    for (int j = 0; j < 10; j++) {
      a.c[i + j] += (uint64_t)x.l[i] * y.l[j];
      asm("" : "+v"(a.c[i + j]));
    }
    acc_redc_digit(a, i);
  }
}
// Montgomery REDC: r = T * 2^-286 mod p, canonical. Requires T < p R
// (11 digits of 26 bits; the result T / R + q p / R < 2p before the final
// conditional subtraction). FROM: digits already done (acc_mad_redc).
template <int FROM = 0>
HG_DEV void acc_reduce(Fp& r, Acc& a) {
  acc_redc_digits<FROM>(a);
  uint32_t x[10];
  acc_redc_limbs(x, a);
  fp_csub_rare(r, x);
}

HG_DEV void fp_mul(Fp& r, const Fp& a, const Fp& b) {
  Acc t;
  acc_zero(t);
  acc_mad(t, a, b);
  acc_reduce(r, t);
}
HG_DEV void fp_sqr(Fp& r, const Fp& a) {
  Acc t;
  acc_zero(t);
  acc_sqr(t, a);
  acc_reduce(r, t);
}

// ---------------------------------------------------------------- add / sub
// loose sum: limb-wise, no carry or reduction (value < 2p, limbs < 2^27)
HG_DEV void fp_add_loose(Fp& r, const Fp& a, const Fp& b) {
#pragma unroll
  for (int i = 0; i < 10; i++) r.l[i] = a.l[i] + b.l[i];
}
HG_DEV void fp_add(Fp& r, const Fp& a, const Fp& b) {
  uint32_t x[10];
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 10; i++) {
    uint32_t v = a.l[i] + b.l[i] + c;
    x[i] = (i < 9) ? (v & kMask) : v;
    c = v >> 26;
  }
  fp_csub(r, x);
}
// r = a - b mod p for reduced a, b
HG_DEV void fp_sub(Fp& r, const Fp& a, const Fp& b) {
  uint32_t x[10];
  int32_t c = 0;
#pragma unroll
  for (int i = 0; i < 10; i++) {
    int32_t v = (int32_t)a.l[i] - (int32_t)b.l[i] + (int32_t)p_limb(i) + c;
    x[i] = (i < 9) ? ((uint32_t)v & kMask) : (uint32_t)v;
    c = v >> 26;  // arithmetic shift: -1, 0 or 1
  }
  fp_csub(r, x);  // a - b + p in (0, 2p)
}
// p - a for reduced a: a value in [1, p] (not canonical when a == 0; fine as a
// multiplication operand)
HG_DEV void fp_neg_loose(Fp& r, const Fp& a) {
  int32_t c = 0;
#pragma unroll
  for (int i = 0; i < 10; i++) {
    int32_t v = (int32_t)p_limb(i) - (int32_t)a.l[i] + c;
    r.l[i] = (i < 9) ? ((uint32_t)v & kMask) : (uint32_t)v;
    c = v >> 26;
  }
}
HG_DEV void fp_neg(Fp& r, const Fp& a) {
  Fp z;
  fp_zero(z);
  fp_sub(r, z, a);
}
HG_DEV void fp_dbl(Fp& r, const Fp& a) { fp_add(r, a, a); }
HG_DEV void fp_mul3(Fp& r, const Fp& a) {
  Fp t;
  fp_add(t, a, a);
  fp_add(r, t, a);
}
// normalize a loose value < 2p (limbs < 2^32) into a canonical element
HG_DEV void fp_norm(Fp& r, const Fp& a) {
  uint32_t x[10];
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 10; i++) {
    uint32_t v = a.l[i] + c;
    x[i] = (i < 9) ? (v & kMask) : v;
    c = v >> 26;
  }
  fp_csub(r, x);
}

// ---------------------------------------------------------------- conversions
// 8 LE 32-bit words (a plain integer < 2^256) -> 10 x 26-bit limbs (no reduction)
HG_DEV void words_to_limbs(Fp& r, const uint32_t* w) {
#pragma unroll
  for (int i = 0; i < 10; i++) {
    int bit = 26 * i;
    int wi = bit >> 5, sh = bit & 31;
    uint64_t v = (uint64_t)w[wi] >> sh;
    if (wi + 1 < 8) v |= (uint64_t)w[wi + 1] << (32 - sh);
    r.l[i] = (uint32_t)v & kMask;
  }
}
HG_DEV void limbs_to_words(uint32_t* w, const Fp& a) {
#pragma unroll
  for (int k = 0; k < 8; k++) w[k] = 0;
#pragma unroll
  for (int i = 0; i < 10; i++) {
    int bit = 26 * i;
    int wi = bit >> 5, sh = bit & 31;
    w[wi] |= a.l[i] << sh;
    if (wi + 1 < 8 && sh > 6) w[wi + 1] |= a.l[i] >> (32 - sh);
  }
}
// plain integer limbs (value < 2^256 < 2p) -> Montgomery form, canonical
HG_DEV void fp_to_mont(Fp& r, const Fp& x) {
  const Fp r2 = {{HG_R2}};
  fp_mul(r, x, r2);
}
HG_DEV void fp_from_mont(Fp& r, const Fp& a) {
  Fp one;
  fp_zero(one);
  one.l[0] = 1;
  fp_mul(r, a, one);
}
// a^-1 for canonical a (0 -> 0): the plain integer inverse of the Montgomery
// representative aR (Bernstein-Yang, bn256_inv.h), times R^3 by one Montgomery
// product: (aR)^-1 R^3 / R = a^-1 R. Replaces the a^(p-2) chain of x/crypto's
// gfP.Invert with an equal result.
HG_DEV void fp_inv(Fp& r, const Fp& a) {
  uint32_t w[8];
  limbs_to_words(w, a);
  inv::inv_words(w);
  Fp x;
  words_to_limbs(x, w);
  const Fp r3 = {{HG_R3}};
  fp_mul(r, x, r3);
}
// big-endian 32 bytes -> LE words; returns true when the value is >= p
HG_DEV bool be_to_words(uint32_t* w, const uint8_t* b) {
  if ((reinterpret_cast<uintptr_t>(b) & 3) == 0) {
    // the marshals' usual case (32-byte coordinates at 4-byte aligned
    // offsets): eight dword loads instead of 32 byte loads
    const uint32_t* q = reinterpret_cast<const uint32_t*>(b);
#pragma unroll
    for (int i = 0; i < 8; i++) w[i] = __builtin_bswap32(q[7 - i]);
  } else {
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const uint8_t* q = b + (7 - i) * 4;
      w[i] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | q[3];
    }
  }
  const uint32_t pw[8] = {HG_P32};
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t d = (uint64_t)w[i] - pw[i] - br;
    br = (uint32_t)(d >> 63);
  }
  return br == 0;
}
HG_DEV void words_to_be(uint8_t* b, const uint32_t* w) {
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint8_t* q = b + (7 - i) * 4;
    q[0] = (uint8_t)(w[i] >> 24);
    q[1] = (uint8_t)(w[i] >> 16);
    q[2] = (uint8_t)(w[i] >> 8);
    q[3] = (uint8_t)w[i];
  }
}
// decode 32 BE bytes into a Montgomery element (value taken mod p); *ge_p set
// when the encoded integer is >= p (cloudflare rejects those)
// nz_p (optional): OR-ed with "some byte of the coordinate is nonzero"
HG_DEV void fp_from_be(Fp& r, const uint8_t* b, bool* ge_p, bool* nz_p = nullptr) {
  uint32_t w[8];
  *ge_p = be_to_words(w, b);
  if (nz_p) {
    uint32_t any = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) any |= w[i];
    *nz_p |= any != 0;
  }
  Fp x;
  words_to_limbs(x, w);
  fp_to_mont(r, x);
}
HG_DEV void fp_to_be(uint8_t* b, const Fp& a) {
  Fp x;
  fp_from_mont(x, a);
  uint32_t w[8];
  limbs_to_words(w, x);
  words_to_be(b, w);
}

// ---------------------------------------------------------------- Fp2 = x*i + y
struct Fp2 {
  Fp x, y;
};

HG_DEV void f2_zero(Fp2& r) { fp_zero(r.x); fp_zero(r.y); }
HG_DEV void f2_one(Fp2& r) { fp_zero(r.x); fp_one(r.y); }
HG_DEV bool f2_is_zero(const Fp2& a) { return fp_is_zero(a.x) && fp_is_zero(a.y); }
HG_DEV bool f2_eq(const Fp2& a, const Fp2& b) { return fp_eq(a.x, b.x) && fp_eq(a.y, b.y); }
HG_DEV void f2_add(Fp2& r, const Fp2& a, const Fp2& b) { fp_add(r.x, a.x, b.x); fp_add(r.y, a.y, b.y); }
HG_DEV void f2_sub(Fp2& r, const Fp2& a, const Fp2& b) { fp_sub(r.x, a.x, b.x); fp_sub(r.y, a.y, b.y); }
HG_DEV void f2_neg(Fp2& r, const Fp2& a) { fp_neg(r.x, a.x); fp_neg(r.y, a.y); }
HG_DEV void f2_dbl(Fp2& r, const Fp2& a) { f2_add(r, a, a); }
HG_DEV void f2_conj(Fp2& r, const Fp2& a) { fp_neg(r.x, a.x); r.y = a.y; }
HG_DEV void f2_sel(Fp2& r, bool c, const Fp2& a, const Fp2& b) {
  fp_sel(r.x, c, a.x, b.x);
  fp_sel(r.y, c, a.y, b.y);
}

// (ax i + ay)(bx i + by) = (ax by + ay bx) i + (ay by - ax bx)
// schoolbook with lazy reduction: 4 products, 2 reductions
HG_DEV void f2_mul(Fp2& r, const Fp2& a, const Fp2& b) {
  Fp nax;
  fp_neg_loose(nax, a.x);
  Acc re, im;
  acc_zero(re);
  acc_zero(im);
  acc_mad(re, a.y, b.y);
  acc_mad(re, nax, b.x);
  acc_mad(im, a.x, b.y);
  acc_mad(im, a.y, b.x);
  acc_reduce(r.y, re);
  acc_reduce(r.x, im);
}
// (x i + y)^2 = 2xy i + (y + x)(y - x)
HG_DEV void f2_sqr(Fp2& r, const Fp2& a) {
  Fp s, d, x2;
  fp_add_loose(s, a.y, a.x);
  fp_sub(d, a.y, a.x);
  fp_add_loose(x2, a.x, a.x);
  Acc re, im;
  acc_zero(re);
  acc_zero(im);
  acc_mad(re, s, d);
  acc_mad(im, x2, a.y);
  acc_reduce(r.y, re);
  acc_reduce(r.x, im);
}
HG_DEV void f2_muls(Fp2& r, const Fp2& a, const Fp& s) {
  fp_mul(r.x, a.x, s);
  fp_mul(r.y, a.y, s);
}
// (x i + y)(i + 3) = (3x + y) i + (3y - x)
HG_DEV void f2_mul_xi(Fp2& r, const Fp2& a) {
  Fp x3, y3, nx, ny;
  fp_mul3(x3, a.x);
  fp_mul3(y3, a.y);
  fp_add(nx, x3, a.y);
  fp_sub(ny, y3, a.x);
  r.x = nx;
  r.y = ny;
}
HG_DEV void f2_inv(Fp2& r, const Fp2& a) {
  Acc t;
  acc_zero(t);
  acc_sqr(t, a.x);
  acc_sqr(t, a.y);
  Fp n;
  acc_reduce(n, t);
  fp_inv(n, n);
  Fp nx;
  fp_neg(nx, a.x);
  fp_mul(r.x, nx, n);
  fp_mul(r.y, a.y, n);
}

}  // namespace hg
