// bn256_curve.h — G1 / G2 group law and optimal-ate line functions, one
// thread per point (used for decode, hash-to-G1, aggregation, affine
// conversion and the per-lane Miller-loop line evaluation).
//
// Group law: Jacobian coordinates with the add-2007-bl / dbl-2009-l formulas
// and the same exceptional-case handling as golang.org/x/crypto/bn256
// curve.go/twist.go (equal inputs -> double, opposite inputs -> infinity),
// so every result is the exact group element the reference's G1.Add /
// G2.Add (bn256/go/bn256.go:103,198) would marshal.
//
// Line functions restate x/crypto optate.go lineFunctionDouble /
// lineFunctionAdd; the line is (a*tau + b)*omega + c = c + b*w + a*w^3.
#pragma once
#include "bn256_fp.h"

namespace hg {

struct G1J {
  Fp x, y, z;
};
struct G2J {
  Fp2 x, y, z;
};
// twist point as used by the Miller loop: T = Z^2
struct G2T {
  Fp2 x, y, z, t;
};

HG_DEV void g1_set_inf(G1J& a) {
  fp_one(a.x);
  fp_one(a.y);
  fp_zero(a.z);
}
HG_DEV bool g1_is_inf(const G1J& a) { return fp_is_zero(a.z); }
HG_DEV void g2_set_inf(G2J& a) {
  f2_one(a.x);
  f2_one(a.y);
  f2_zero(a.z);
}
HG_DEV bool g2_is_inf(const G2J& a) { return f2_is_zero(a.z); }

// ----------------------------------------------------------------- G1
HG_DEV void g1_double(G1J& r, const G1J& a) {
  if (g1_is_inf(a)) {
    r = a;
    return;
  }
  Fp A, B, C, D, E, F, t, x3, y3, z3;
  fp_sqr(A, a.x);
  fp_sqr(B, a.y);
  fp_sqr(C, B);
  fp_add(t, a.x, B);
  fp_sqr(D, t);
  fp_sub(D, D, A);
  fp_sub(D, D, C);
  fp_dbl(D, D);
  fp_mul3(E, A);
  fp_sqr(F, E);
  fp_dbl(t, D);
  fp_sub(x3, F, t);
  fp_dbl(t, C);
  fp_dbl(t, t);
  fp_dbl(t, t);
  fp_sub(y3, D, x3);
  fp_mul(y3, E, y3);
  fp_sub(y3, y3, t);
  fp_mul(z3, a.y, a.z);
  fp_dbl(z3, z3);
  r.x = x3;
  r.y = y3;
  r.z = z3;
}

HG_DEV void g1_add(G1J& r, const G1J& a, const G1J& b) {
  if (g1_is_inf(a)) {
    r = b;
    return;
  }
  if (g1_is_inf(b)) {
    r = a;
    return;
  }
  Fp z1z1, z2z2, u1, u2, s1, s2, h, rr, i, j, v, t, x3, y3, z3;
  fp_sqr(z1z1, a.z);
  fp_sqr(z2z2, b.z);
  fp_mul(u1, a.x, z2z2);
  fp_mul(u2, b.x, z1z1);
  fp_mul(t, b.z, z2z2);
  fp_mul(s1, a.y, t);
  fp_mul(t, a.z, z1z1);
  fp_mul(s2, b.y, t);
  fp_sub(h, u2, u1);
  fp_sub(rr, s2, s1);
  if (fp_is_zero(h)) {
    if (fp_is_zero(rr)) {
      g1_double(r, a);
    } else {
      g1_set_inf(r);
    }
    return;
  }
  fp_dbl(t, h);
  fp_sqr(i, t);
  fp_mul(j, h, i);
  fp_dbl(rr, rr);
  fp_mul(v, u1, i);
  fp_sqr(x3, rr);
  fp_sub(x3, x3, j);
  fp_sub(x3, x3, v);
  fp_sub(x3, x3, v);
  fp_sub(t, v, x3);
  fp_mul(y3, rr, t);
  fp_mul(t, s1, j);
  fp_dbl(t, t);
  fp_sub(y3, y3, t);
  fp_add(t, a.z, b.z);
  fp_sqr(t, t);
  fp_sub(t, t, z1z1);
  fp_sub(t, t, z2z2);
  fp_mul(z3, t, h);
  r.x = x3;
  r.y = y3;
  r.z = z3;
}

// k * a for a 256-bit scalar given as 8 LE 32-bit words (double-and-add, MSB first)
HG_DEV void g1_mul(G1J& r, const G1J& a, const uint32_t* k) {
  G1J acc;
  g1_set_inf(acc);
  for (int i = 7; i >= 0; i--) {
    for (int bit = 31; bit >= 0; bit--) {
      g1_double(acc, acc);
      if ((k[i] >> bit) & 1) g1_add(acc, acc, a);
    }
  }
  r = acc;
}

HG_DEV void g1_affine(Fp& x, Fp& y, const G1J& a) {
  Fp zi, zi2, zi3;
  fp_inv(zi, a.z);
  fp_sqr(zi2, zi);
  fp_mul(zi3, zi2, zi);
  fp_mul(x, a.x, zi2);
  fp_mul(y, a.y, zi3);
}

HG_DEV bool g1_on_curve(const Fp& x, const Fp& y) {
  const Fp b = HG_CURVE_B;
  Fp yy, xxx;
  fp_sqr(yy, y);
  fp_sqr(xxx, x);
  fp_mul(xxx, xxx, x);
  fp_add(xxx, xxx, b);
  return fp_eq(yy, xxx);
}

// ----------------------------------------------------------------- G2
HG_DEV void g2_double(G2J& r, const G2J& a) {
  if (g2_is_inf(a)) {
    r = a;
    return;
  }
  Fp2 A, B, C, D, E, F, t, x3, y3, z3;
  f2_sqr(A, a.x);
  f2_sqr(B, a.y);
  f2_sqr(C, B);
  f2_add(t, a.x, B);
  f2_sqr(D, t);
  f2_sub(D, D, A);
  f2_sub(D, D, C);
  f2_dbl(D, D);
  f2_add(E, A, A);
  f2_add(E, E, A);
  f2_sqr(F, E);
  f2_dbl(t, D);
  f2_sub(x3, F, t);
  f2_dbl(t, C);
  f2_dbl(t, t);
  f2_dbl(t, t);
  f2_sub(y3, D, x3);
  f2_mul(y3, E, y3);
  f2_sub(y3, y3, t);
  f2_mul(z3, a.y, a.z);
  f2_dbl(z3, z3);
  r.x = x3;
  r.y = y3;
  r.z = z3;
}

HG_DEV void g2_add(G2J& r, const G2J& a, const G2J& b) {
  if (g2_is_inf(a)) {
    r = b;
    return;
  }
  if (g2_is_inf(b)) {
    r = a;
    return;
  }
  Fp2 z1z1, z2z2, u1, u2, s1, s2, h, rr, i, j, v, t, x3, y3, z3;
  f2_sqr(z1z1, a.z);
  f2_sqr(z2z2, b.z);
  f2_mul(u1, a.x, z2z2);
  f2_mul(u2, b.x, z1z1);
  f2_mul(t, b.z, z2z2);
  f2_mul(s1, a.y, t);
  f2_mul(t, a.z, z1z1);
  f2_mul(s2, b.y, t);
  f2_sub(h, u2, u1);
  f2_sub(rr, s2, s1);
  if (f2_is_zero(h)) {
    if (f2_is_zero(rr)) {
      g2_double(r, a);
    } else {
      g2_set_inf(r);
    }
    return;
  }
  f2_dbl(t, h);
  f2_sqr(i, t);
  f2_mul(j, h, i);
  f2_dbl(rr, rr);
  f2_mul(v, u1, i);
  f2_sqr(x3, rr);
  f2_sub(x3, x3, j);
  f2_sub(x3, x3, v);
  f2_sub(x3, x3, v);
  f2_sub(t, v, x3);
  f2_mul(y3, rr, t);
  f2_mul(t, s1, j);
  f2_dbl(t, t);
  f2_sub(y3, y3, t);
  f2_add(t, a.z, b.z);
  f2_sqr(t, t);
  f2_sub(t, t, z1z1);
  f2_sub(t, t, z2z2);
  f2_mul(z3, t, h);
  r.x = x3;
  r.y = y3;
  r.z = z3;
}

// mixed addition a + (bx, by) with b affine (madd-2007-bl: 7M + 4S instead of
// the 11M + 5S of g2_add with z = 1); a at infinity, a == b (doubling) and
// a == -b (infinity) handled as in g2_add. Used by the aggregation fold.
HG_DEV void g2_madd(G2J& r, const G2J& a, const Fp2& bx, const Fp2& by) {
  if (g2_is_inf(a)) {
    r.x = bx;
    r.y = by;
    f2_one(r.z);
    return;
  }
  Fp2 z1z1, u2, s2, h, hh, i, j, rr, v, t, x3, y3, z3;
  f2_sqr(z1z1, a.z);
  f2_mul(u2, bx, z1z1);
  f2_mul(t, a.z, z1z1);
  f2_mul(s2, by, t);
  f2_sub(h, u2, a.x);
  f2_sub(rr, s2, a.y);
  if (f2_is_zero(h)) {
    if (f2_is_zero(rr)) {
      g2_double(r, a);
    } else {
      g2_set_inf(r);
    }
    return;
  }
  f2_sqr(hh, h);
  f2_dbl(i, hh);
  f2_dbl(i, i);
  f2_mul(j, h, i);
  f2_dbl(rr, rr);
  f2_mul(v, a.x, i);
  f2_sqr(x3, rr);
  f2_sub(x3, x3, j);
  f2_sub(x3, x3, v);
  f2_sub(x3, x3, v);
  f2_sub(t, v, x3);
  f2_mul(y3, rr, t);
  f2_mul(t, a.y, j);
  f2_dbl(t, t);
  f2_sub(y3, y3, t);
  f2_add(t, a.z, h);
  f2_sqr(t, t);
  f2_sub(t, t, z1z1);
  f2_sub(z3, t, hh);
  r.x = x3;
  r.y = y3;
  r.z = z3;
}

// mixed add: b affine (z = 1), full exceptional-case handling
HG_DEV void g2_add_affine(G2J& r, const G2J& a, const Fp2& bx, const Fp2& by) {
  G2J b;
  b.x = bx;
  b.y = by;
  f2_one(b.z);
  g2_add(r, a, b);
}

HG_DEV void g2_mul(G2J& r, const G2J& a, const uint32_t* k) {
  G2J acc;
  g2_set_inf(acc);
  for (int i = 7; i >= 0; i--) {
    for (int bit = 31; bit >= 0; bit--) {
      g2_double(acc, acc);
      if ((k[i] >> bit) & 1) g2_add(acc, acc, a);
    }
  }
  r = acc;
}

HG_DEV void g2_affine(Fp2& x, Fp2& y, const G2J& a) {
  Fp2 zi, zi2, zi3;
  f2_inv(zi, a.z);
  f2_sqr(zi2, zi);
  f2_mul(zi3, zi2, zi);
  f2_mul(x, a.x, zi2);
  f2_mul(y, a.y, zi3);
}

HG_DEV bool g2_on_curve(const Fp2& x, const Fp2& y) {
  const Fp2 b = HG_TWIST_B;
  Fp2 yy, xxx;
  f2_sqr(yy, y);
  f2_sqr(xxx, x);
  f2_mul(xxx, xxx, x);
  f2_add(xxx, xxx, b);
  return f2_eq(yy, xxx);
}

// ----------------------------------------------------------------- lines
// x/crypto optate.go lineFunctionDouble: doubles r in place and returns the
// line coefficients; bx/cy are the parts that get multiplied by the G1
// point's x and y (b = bx * Px, c = cy * Py).
HG_DEV void line_double(Fp2& a, Fp2& bx, Fp2& cy, G2T& r) {
  Fp2 A, B, C, D, E, G, t, xo, yo, zo, to;
  f2_sqr(A, r.x);
  f2_sqr(B, r.y);
  f2_sqr(C, B);
  f2_add(D, r.x, B);
  f2_sqr(D, D);
  f2_sub(D, D, A);
  f2_sub(D, D, C);
  f2_dbl(D, D);
  f2_add(E, A, A);
  f2_add(E, E, A);
  f2_sqr(G, E);
  f2_sub(xo, G, D);
  f2_sub(xo, xo, D);
  f2_add(zo, r.y, r.z);
  f2_sqr(zo, zo);
  f2_sub(zo, zo, B);
  f2_sub(zo, zo, r.t);
  f2_sub(yo, D, xo);
  f2_mul(yo, yo, E);
  f2_dbl(t, C);
  f2_dbl(t, t);
  f2_dbl(t, t);
  f2_sub(yo, yo, t);
  f2_sqr(to, zo);
  f2_mul(t, E, r.t);
  f2_dbl(t, t);
  f2_neg(bx, t);  // b = -2 E T * Px
  f2_add(a, r.x, E);
  f2_sqr(a, a);
  f2_sub(a, a, A);
  f2_sub(a, a, G);
  f2_dbl(t, B);
  f2_dbl(t, t);
  f2_sub(a, a, t);
  f2_mul(cy, zo, r.t);
  f2_dbl(cy, cy);  // c = 2 Z' T * Py
  r.x = xo;
  r.y = yo;
  r.z = zo;
  r.t = to;
}

// x/crypto optate.go lineFunctionAdd: r += (px, py) (affine), r2 = py^2
HG_DEV void line_add(Fp2& a, Fp2& bx, Fp2& cy, G2T& r, const Fp2& px, const Fp2& py, const Fp2& r2) {
  Fp2 B, D, H, I, E, J, L1, V, t, t2, xo, yo, zo, to;
  f2_mul(B, px, r.t);
  f2_add(D, py, r.z);
  f2_sqr(D, D);
  f2_sub(D, D, r2);
  f2_sub(D, D, r.t);
  f2_mul(D, D, r.t);
  f2_sub(H, B, r.x);
  f2_sqr(I, H);
  f2_dbl(E, I);
  f2_dbl(E, E);
  f2_mul(J, H, E);
  f2_sub(L1, D, r.y);
  f2_sub(L1, L1, r.y);
  f2_mul(V, r.x, E);
  f2_sqr(xo, L1);
  f2_sub(xo, xo, J);
  f2_sub(xo, xo, V);
  f2_sub(xo, xo, V);
  f2_add(zo, r.z, H);
  f2_sqr(zo, zo);
  f2_sub(zo, zo, r.t);
  f2_sub(zo, zo, I);
  f2_sub(t, V, xo);
  f2_mul(t, t, L1);
  f2_mul(t2, r.y, J);
  f2_dbl(t2, t2);
  f2_sub(yo, t, t2);
  f2_sqr(to, zo);
  f2_add(t, py, zo);
  f2_sqr(t, t);
  f2_sub(t, t, r2);
  f2_sub(t, t, to);
  f2_mul(t2, L1, px);
  f2_dbl(t2, t2);
  f2_sub(a, t2, t);
  f2_dbl(cy, zo);   // c = 2 Z' * Py
  f2_dbl(bx, L1);
  f2_neg(bx, bx);   // b = -2 L1 * Px
  r.x = xo;
  r.y = yo;
  r.z = zo;
  r.t = to;
}

}  // namespace hg
