// bn256_inv.h — variable-time modular inversion mod p by Bernstein–Yang
// divsteps ("safegcd"; batches of 30 divsteps on 32-bit words on the device
// path, the 62-divstep 64-bit form kept beside it), the
// inversion behind fp_inv (final exponentiation's Fp6 norm inverse, affine
// conversions).
//
// The reference computes the same inverse as a^(p-2) (x/crypto gfP.Invert,
// a Fermat exponentiation: 255 squarings + ~128 multiplications, one
// dependent chain). Inputs on the verification path are public (signatures,
// keys, pairing values), so a variable-time gcd is acceptable, and it is an
// order of magnitude shorter: ~10 batches of 62 divsteps, each batch a loop of
// 64-bit word operations plus one 2x2 matrix application to 5-limb numbers.
//
// Numbers are "signed62": 5 signed 64-bit limbs of 62 bits (310 bits). The
// structure follows the published safegcd algorithm (Bernstein & Yang 2019,
// "Fast constant-time gcd computation and modular inversion", §11, with the
// variable-time batching of divsteps by trailing-zero counts).
//
// Host-compilable (HG_HD) so tests/ can check it against Python's pow(a, -1, p).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define HG_HD __host__ __device__ inline
#else
#define HG_HD static inline
#endif

namespace hg {
namespace inv {

struct S62 {
  int64_t v[5];
};
struct Mat {
  int64_t u, v, q, r;
};

static constexpr uint64_t kM62 = UINT64_MAX >> 2;

// p in signed62 limbs and p^-1 mod 2^62
#define HG_P62 0x185cac6c5e089667ll, 0x396e234482d6d678ll, 0x26fecb86184dc21ell, 0x2d4078d2a8e1fe6all, 0x8fll
static constexpr uint64_t kPInv62 = 0x1c7806ff80e82557ull;  // p^-1 mod 2^62 (tests check p * inv == 1)

HG_HD int ctz64(uint64_t x) { return __builtin_ctzll(x); }

// 62 divsteps on the low words of f, g (eta = -delta); returns the new eta
// and the transition matrix scaled by 2^62.
HG_HD int64_t divsteps_62_var(int64_t eta, uint64_t f0, uint64_t g0, Mat* t) {
  uint64_t u = 1, v = 0, q = 0, r = 1;
  uint64_t f = f0, g = g0, m;
  uint32_t w;
  int i = 62, limit, zeros;
  for (;;) {
    // a sentinel bit limits the count to the i steps left
    zeros = ctz64(g | (UINT64_MAX << i));
    g >>= zeros;
    u <<= zeros;
    v <<= zeros;
    eta -= zeros;
    i -= zeros;
    if (i == 0) break;
    if (eta < 0) {
      // swap f, g (g = -f) and cancel up to 6 low bits of g
      uint64_t tmp;
      eta = -eta;
      tmp = f; f = g; g = (uint64_t)0 - tmp;
      tmp = u; u = q; q = (uint64_t)0 - tmp;
      tmp = v; v = r; r = (uint64_t)0 - tmp;
      limit = ((int)eta + 1) > i ? i : ((int)eta + 1);
      m = (UINT64_MAX >> (64 - limit)) & 63u;
      w = (uint32_t)((f * g * (f * f - 2)) & m);
    } else {
      // cancel up to 4 low bits of g
      limit = ((int)eta + 1) > i ? i : ((int)eta + 1);
      m = (UINT64_MAX >> (64 - limit)) & 15u;
      w = (uint32_t)(f + (((f + 1) & 4) << 1));
      w = (uint32_t)(((uint64_t)0 - (uint64_t)w * g) & m);
    }
    g += f * w;
    q += u * w;
    r += v * w;
  }
  t->u = (int64_t)u;
  t->v = (int64_t)v;
  t->q = (int64_t)q;
  t->r = (int64_t)r;
  return eta;
}

// [d, e] <- t [d, e] / 2^62 (mod p), keeping d, e in (-2p, p)
HG_HD void update_de_62(S62* d, S62* e, const Mat* t) {
  const int64_t P[5] = {HG_P62};
  const int64_t d0 = d->v[0], d1 = d->v[1], d2 = d->v[2], d3 = d->v[3], d4 = d->v[4];
  const int64_t e0 = e->v[0], e1 = e->v[1], e2 = e->v[2], e3 = e->v[3], e4 = e->v[4];
  const int64_t u = t->u, v = t->v, q = t->q, r = t->r;
  int64_t md, me, sd, se;
  __int128 cd, ce;
  sd = d4 >> 63;
  se = e4 >> 63;
  md = (u & sd) + (v & se);
  me = (q & sd) + (r & se);
  cd = (__int128)u * d0 + (__int128)v * e0;
  ce = (__int128)q * d0 + (__int128)r * e0;
  // choose md, me so that the low 62 bits of t [d, e] + p [md, me] vanish
  md -= (int64_t)((kPInv62 * (uint64_t)cd + (uint64_t)md) & kM62);
  me -= (int64_t)((kPInv62 * (uint64_t)ce + (uint64_t)me) & kM62);
  cd += (__int128)P[0] * md;
  ce += (__int128)P[0] * me;
  cd >>= 62;
  ce >>= 62;
  cd += (__int128)u * d1 + (__int128)v * e1 + (__int128)P[1] * md;
  ce += (__int128)q * d1 + (__int128)r * e1 + (__int128)P[1] * me;
  d->v[0] = (int64_t)((uint64_t)cd & kM62);
  cd >>= 62;
  e->v[0] = (int64_t)((uint64_t)ce & kM62);
  ce >>= 62;
  cd += (__int128)u * d2 + (__int128)v * e2 + (__int128)P[2] * md;
  ce += (__int128)q * d2 + (__int128)r * e2 + (__int128)P[2] * me;
  d->v[1] = (int64_t)((uint64_t)cd & kM62);
  cd >>= 62;
  e->v[1] = (int64_t)((uint64_t)ce & kM62);
  ce >>= 62;
  cd += (__int128)u * d3 + (__int128)v * e3 + (__int128)P[3] * md;
  ce += (__int128)q * d3 + (__int128)r * e3 + (__int128)P[3] * me;
  d->v[2] = (int64_t)((uint64_t)cd & kM62);
  cd >>= 62;
  e->v[2] = (int64_t)((uint64_t)ce & kM62);
  ce >>= 62;
  cd += (__int128)u * d4 + (__int128)v * e4 + (__int128)P[4] * md;
  ce += (__int128)q * d4 + (__int128)r * e4 + (__int128)P[4] * me;
  d->v[3] = (int64_t)((uint64_t)cd & kM62);
  cd >>= 62;
  e->v[3] = (int64_t)((uint64_t)ce & kM62);
  ce >>= 62;
  d->v[4] = (int64_t)cd;
  e->v[4] = (int64_t)ce;
}

// [f, g] <- t [f, g] / 2^62 (exact), on the low len limbs
HG_HD void update_fg_62_var(int len, S62* f, S62* g, const Mat* t) {
  const int64_t u = t->u, v = t->v, q = t->q, r = t->r;
  int64_t fi, gi;
  __int128 cf, cg;
  fi = f->v[0];
  gi = g->v[0];
  cf = (__int128)u * fi + (__int128)v * gi;
  cg = (__int128)q * fi + (__int128)r * gi;
  cf >>= 62;
  cg >>= 62;
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
  for (int i = 1; i < len; ++i) {
    fi = f->v[i];
    gi = g->v[i];
    cf += (__int128)u * fi + (__int128)v * gi;
    cg += (__int128)q * fi + (__int128)r * gi;
    f->v[i - 1] = (int64_t)((uint64_t)cf & kM62);
    cf >>= 62;
    g->v[i - 1] = (int64_t)((uint64_t)cg & kM62);
    cg >>= 62;
  }
  f->v[len - 1] = (int64_t)cf;
  g->v[len - 1] = (int64_t)cg;
}

// r in (-2p, p) -> r * sign(sign) mod p in [0, p)
HG_HD void normalize_62(S62* r, int64_t sign) {
  const int64_t P[5] = {HG_P62};
  const int64_t M62 = (int64_t)kM62;
  int64_t r0 = r->v[0], r1 = r->v[1], r2 = r->v[2], r3 = r->v[3], r4 = r->v[4];
  int64_t cond_add, cond_negate;
  cond_add = r4 >> 63;
  r0 += P[0] & cond_add;
  r1 += P[1] & cond_add;
  r2 += P[2] & cond_add;
  r3 += P[3] & cond_add;
  r4 += P[4] & cond_add;
  cond_negate = sign >> 63;
  r0 = (r0 ^ cond_negate) - cond_negate;
  r1 = (r1 ^ cond_negate) - cond_negate;
  r2 = (r2 ^ cond_negate) - cond_negate;
  r3 = (r3 ^ cond_negate) - cond_negate;
  r4 = (r4 ^ cond_negate) - cond_negate;
  r1 += r0 >> 62;
  r0 &= M62;
  r2 += r1 >> 62;
  r1 &= M62;
  r3 += r2 >> 62;
  r2 &= M62;
  r4 += r3 >> 62;
  r3 &= M62;
  cond_add = r4 >> 63;
  r0 += P[0] & cond_add;
  r1 += P[1] & cond_add;
  r2 += P[2] & cond_add;
  r3 += P[3] & cond_add;
  r4 += P[4] & cond_add;
  r1 += r0 >> 62;
  r0 &= M62;
  r2 += r1 >> 62;
  r1 &= M62;
  r3 += r2 >> 62;
  r2 &= M62;
  r4 += r3 >> 62;
  r3 &= M62;
  r->v[0] = r0;
  r->v[1] = r1;
  r->v[2] = r2;
  r->v[3] = r3;
  r->v[4] = r4;
}

// x <- x^-1 mod p for 0 <= x < p (0 -> 0). All five limbs of f and g are
// always updated (no length shortening): every limb index is a constant after
// unrolling, so the device code keeps f, g, d, e in registers.
HG_HD void modinv_var(S62* x) {
  const int64_t P[5] = {HG_P62};
  S62 d = {{0, 0, 0, 0, 0}};
  S62 e = {{1, 0, 0, 0, 0}};
  S62 f = {{P[0], P[1], P[2], P[3], P[4]}};
  S62 g = *x;
  int64_t eta = -1;  // eta = -delta, delta = 1
  for (;;) {
    Mat t;
    eta = divsteps_62_var(eta, (uint64_t)f.v[0], (uint64_t)g.v[0], &t);
    update_de_62(&d, &e, &t);
    update_fg_62_var(5, &f, &g, &t);
    if ((g.v[0] | g.v[1] | g.v[2] | g.v[3] | g.v[4]) == 0) break;
  }
  normalize_62(&d, f.v[4]);
  *x = d;
}

// 8 LE 32-bit words <-> signed62
HG_HD void words_to_s62(S62* r, const uint32_t* w) {
  uint64_t a0 = w[0] | ((uint64_t)w[1] << 32), a1 = w[2] | ((uint64_t)w[3] << 32);
  uint64_t a2 = w[4] | ((uint64_t)w[5] << 32), a3 = w[6] | ((uint64_t)w[7] << 32);
  r->v[0] = (int64_t)(a0 & kM62);
  r->v[1] = (int64_t)(((a0 >> 62) | (a1 << 2)) & kM62);
  r->v[2] = (int64_t)(((a1 >> 60) | (a2 << 4)) & kM62);
  r->v[3] = (int64_t)(((a2 >> 58) | (a3 << 6)) & kM62);
  r->v[4] = (int64_t)(a3 >> 56);
}
HG_HD void s62_to_words(uint32_t* w, const S62* r) {
  const uint64_t v0 = (uint64_t)r->v[0], v1 = (uint64_t)r->v[1], v2 = (uint64_t)r->v[2];
  const uint64_t v3 = (uint64_t)r->v[3], v4 = (uint64_t)r->v[4];
  const uint64_t a0 = v0 | (v1 << 62), a1 = (v1 >> 2) | (v2 << 60), a2 = (v2 >> 4) | (v3 << 58),
                 a3 = (v3 >> 6) | (v4 << 56);
  w[0] = (uint32_t)a0;
  w[1] = (uint32_t)(a0 >> 32);
  w[2] = (uint32_t)a1;
  w[3] = (uint32_t)(a1 >> 32);
  w[4] = (uint32_t)a2;
  w[5] = (uint32_t)(a2 >> 32);
  w[6] = (uint32_t)a3;
  w[7] = (uint32_t)(a3 >> 32);
}

// plain integer inverse on signed62 limbs (kept for comparison; the device
// path uses the signed30 version below)
HG_HD void inv_words62(uint32_t* w) {
  S62 x;
  words_to_s62(&x, w);
  modinv_var(&x);
  s62_to_words(w, &x);
}

// ---------------------------------------------------------------- signed30
// The same algorithm on 32-bit words: batches of 30 divsteps on uint32, a
// transition matrix of int32 entries, and 9-limb signed30 numbers updated with
// int32 x int32 -> int64 multiply-adds (one v_mad_i64_i32 each). On gfx950 the
// 64-bit version's 64x64 -> 128-bit products and 64-bit shifts cost several
// 32-bit instructions each; here every divstep is 32-bit ALU work and every
// matrix product is a native 32x32 -> 64 multiply-add.
struct S30 {
  int32_t v[9];
};
struct Mat30 {
  int32_t u, v, q, r;
};
static constexpr uint32_t kM30 = 0x3fffffffu;
#define HG_P30 0x1e089667, 0x2172b1b1, 0x0b5b59e1, 0x16e23448, 0x04dc21ee, 0x3fb2e186, 0x387f9aa6, 0x0078d2a8, 0x8fb5
static constexpr uint32_t kPInv30 = 0x00e82557u;  // p^-1 mod 2^30 (tests check p * inv == 1)

HG_HD int ctz32(uint32_t x) { return __builtin_ctz(x); }

// 30 divsteps on the low words of f, g (eta = -delta); returns the new eta
// and the transition matrix scaled by 2^30.
HG_HD int32_t divsteps_30_var(int32_t eta, uint32_t f0, uint32_t g0, Mat30* t) {
  uint32_t u = 1, v = 0, q = 0, r = 1;
  uint32_t f = f0, g = g0, m, w;
  int i = 30, limit, zeros;
  for (;;) {
    zeros = ctz32(g | (UINT32_MAX << i));
    g >>= zeros;
    u <<= zeros;
    v <<= zeros;
    eta -= zeros;
    i -= zeros;
    if (i == 0) break;
    if (eta < 0) {
      uint32_t tmp;
      eta = -eta;
      tmp = f; f = g; g = 0u - tmp;
      tmp = u; u = q; q = 0u - tmp;
      tmp = v; v = r; r = 0u - tmp;
      limit = (eta + 1) > i ? i : (eta + 1);
      m = (UINT32_MAX >> (32 - limit)) & 63u;
      w = (f * g * (f * f - 2)) & m;
    } else {
      limit = (eta + 1) > i ? i : (eta + 1);
      m = (UINT32_MAX >> (32 - limit)) & 15u;
      w = f + (((f + 1) & 4) << 1);
      w = (0u - w * g) & m;
    }
    g += f * w;
    q += u * w;
    r += v * w;
  }
  t->u = (int32_t)u;
  t->v = (int32_t)v;
  t->q = (int32_t)q;
  t->r = (int32_t)r;
  return eta;
}

// [d, e] <- t [d, e] / 2^30 (mod p), keeping d, e in (-2p, p)
HG_HD void update_de_30(S30* d, S30* e, const Mat30* t) {
  const int32_t P[9] = {HG_P30};
  const int32_t u = t->u, v = t->v, q = t->q, r = t->r;
  const int32_t sd = d->v[8] >> 31, se = e->v[8] >> 31;
  int32_t md = (u & sd) + (v & se);
  int32_t me = (q & sd) + (r & se);
  int64_t cd = (int64_t)u * d->v[0] + (int64_t)v * e->v[0];
  int64_t ce = (int64_t)q * d->v[0] + (int64_t)r * e->v[0];
  // choose md, me so that the low 30 bits of t [d, e] + p [md, me] vanish
  md -= (int32_t)((kPInv30 * (uint32_t)cd + (uint32_t)md) & kM30);
  me -= (int32_t)((kPInv30 * (uint32_t)ce + (uint32_t)me) & kM30);
  cd += (int64_t)P[0] * md;
  ce += (int64_t)P[0] * me;
  cd >>= 30;
  ce >>= 30;
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
  for (int i = 1; i < 9; i++) {
    cd += (int64_t)u * d->v[i] + (int64_t)v * e->v[i] + (int64_t)P[i] * md;
    ce += (int64_t)q * d->v[i] + (int64_t)r * e->v[i] + (int64_t)P[i] * me;
    d->v[i - 1] = (int32_t)((uint32_t)cd & kM30);
    cd >>= 30;
    e->v[i - 1] = (int32_t)((uint32_t)ce & kM30);
    ce >>= 30;
  }
  d->v[8] = (int32_t)cd;
  e->v[8] = (int32_t)ce;
}

// [f, g] <- t [f, g] / 2^30 (exact), all 9 limbs
HG_HD void update_fg_30(S30* f, S30* g, const Mat30* t) {
  const int32_t u = t->u, v = t->v, q = t->q, r = t->r;
  int64_t cf = (int64_t)u * f->v[0] + (int64_t)v * g->v[0];
  int64_t cg = (int64_t)q * f->v[0] + (int64_t)r * g->v[0];
  cf >>= 30;
  cg >>= 30;
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
  for (int i = 1; i < 9; i++) {
    cf += (int64_t)u * f->v[i] + (int64_t)v * g->v[i];
    cg += (int64_t)q * f->v[i] + (int64_t)r * g->v[i];
    f->v[i - 1] = (int32_t)((uint32_t)cf & kM30);
    cf >>= 30;
    g->v[i - 1] = (int32_t)((uint32_t)cg & kM30);
    cg >>= 30;
  }
  f->v[8] = (int32_t)cf;
  g->v[8] = (int32_t)cg;
}

// r in (-2p, p) -> r * sign(sign) mod p in [0, p)
HG_HD void normalize_30(S30* r, int32_t sign) {
  const int32_t P[9] = {HG_P30};
  int32_t x[9];
  for (int i = 0; i < 9; i++) x[i] = r->v[i];
  int32_t cond_add = x[8] >> 31;
  for (int i = 0; i < 9; i++) x[i] += P[i] & cond_add;
  const int32_t cond_negate = sign >> 31;
  for (int i = 0; i < 9; i++) x[i] = (x[i] ^ cond_negate) - cond_negate;
  for (int i = 0; i < 8; i++) {
    x[i + 1] += x[i] >> 30;
    x[i] &= (int32_t)kM30;
  }
  cond_add = x[8] >> 31;
  for (int i = 0; i < 9; i++) x[i] += P[i] & cond_add;
  for (int i = 0; i < 8; i++) {
    x[i + 1] += x[i] >> 30;
    x[i] &= (int32_t)kM30;
  }
  for (int i = 0; i < 9; i++) r->v[i] = x[i];
}

// x <- x^-1 mod p for 0 <= x < p (0 -> 0)
HG_HD void modinv30_var(S30* x) {
  S30 d = {{0, 0, 0, 0, 0, 0, 0, 0, 0}};
  S30 e = {{1, 0, 0, 0, 0, 0, 0, 0, 0}};
  S30 f = {{HG_P30}};
  S30 g = *x;
  int32_t eta = -1;  // eta = -delta, delta = 1
  for (;;) {
    Mat30 t;
    eta = divsteps_30_var(eta, (uint32_t)f.v[0], (uint32_t)g.v[0], &t);
    update_de_30(&d, &e, &t);
    update_fg_30(&f, &g, &t);
    int32_t z = 0;
    for (int i = 0; i < 9; i++) z |= g.v[i];
    if (z == 0) break;
  }
  normalize_30(&d, f.v[8]);
  *x = d;
}

// 8 LE 32-bit words <-> signed30 (bit 30 k + j of the value = bit j of limb k)
HG_HD void words_to_s30(S30* r, const uint32_t* w) {
  for (int k = 0; k < 9; k++) {
    const int bit = 30 * k, wi = bit >> 5, sh = bit & 31;
    uint64_t v = (uint64_t)w[wi] >> sh;
    if (wi + 1 < 8) v |= (uint64_t)w[wi + 1] << (32 - sh);
    r->v[k] = (int32_t)((uint32_t)v & kM30);
  }
}
HG_HD void s30_to_words(uint32_t* w, const S30* r) {
  for (int i = 0; i < 8; i++) w[i] = 0;
  for (int k = 0; k < 9; k++) {
    const int bit = 30 * k, wi = bit >> 5, sh = bit & 31;
    const uint32_t v = (uint32_t)r->v[k];
    w[wi] |= v << sh;
    if (wi + 1 < 8 && sh > 2) w[wi + 1] |= v >> (32 - sh);
  }
}

// plain integer inverse: w (8 LE words, value < p) <- w^-1 mod p
HG_HD void inv_words(uint32_t* w) {
  S30 x;
  words_to_s30(&x, w);
  modinv30_var(&x);
  s30_to_words(w, &x);
}

}  // namespace inv
}  // namespace hg
