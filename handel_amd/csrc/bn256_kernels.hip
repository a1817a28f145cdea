// bn256_kernels.hip — the HIP kernels of the BN256 BLS verification path.
//
//   k_decode_g2 / k_decode_g1   marshalled points -> affine Montgomery + codes
//                               (x/crypto / cloudflare Unmarshal rules, a9)
//   k_hash_point                k * G1 for the hashedMessage scalar (a7)
//   k_g2_lines                  the fixed G2Base line table (precomputed once)
//   (k_verify: bn256_verify.hip; k_pair and the Fp12 probe: bn256_pair.hip)
//   k_aggregate                 bitset-driven G2 Combine fold, one wave per
//                               request, LDS tree reduction (a3, a4, a5)
//   k_g1_combine                batched SigBLS.Combine (a8)
//   k_fp_mul                    field self-test
#include <cstdlib>
#include <hip/hip_runtime.h>

#include "bn256_kernels.h"
#include "bn256_curve.h"

namespace hg {


// ------------------------------------------------------------------ decode
// Unmarshal rules:
//   go (x/crypto): exact length checked by the host; coordinates taken mod p;
//                  all-zero => infinity; else must be on the curve.
//   cf (cloudflare): each coordinate must be < p; all-zero => infinity; on
//                  the curve; G2 additionally in the order-n subgroup.
__global__ void k_decode_g2(const uint8_t* bytes, int n, int flavor, PointG2* out, int32_t* codes) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint8_t* m = bytes + (size_t)i * 128;
  bool ge[4];
  PointG2 P;
  fp_from_be(P.x.x, m, &ge[0]);
  fp_from_be(P.x.y, m + 32, &ge[1]);
  fp_from_be(P.y.x, m + 64, &ge[2]);
  fp_from_be(P.y.y, m + 96, &ge[3]);
  bool nz = false;
  for (int k = 0; k < 128; k++) nz |= m[k] != 0;
  int32_t code = HG_OK;
  P.inf = nz ? 0u : 1u;
  if (flavor == HG_FLAVOR_CF && (ge[0] || ge[1] || ge[2] || ge[3])) {
    code = HG_ERR_CF_EXCEEDS;
  } else if (nz) {
    if (!g2_on_curve(P.x, P.y)) {
      code = flavor == HG_FLAVOR_CF ? HG_ERR_CF_MALFORMED : HG_ERR_PK_UNMARSHAL;
    } else if (flavor == HG_FLAVOR_CF) {
      // order-n subgroup check (cloudflare twistPoint.IsOnCurve multiplies by Order)
      const uint32_t order[8] = {HG_ORDER32};
      G2J a, r;
      a.x = P.x;
      a.y = P.y;
      f2_one(a.z);
      g2_mul(r, a, order);
      if (!g2_is_inf(r)) code = HG_ERR_CF_MALFORMED;
    }
  }
  out[i] = P;
  codes[i] = code;
}

__global__ void k_decode_g1(const uint8_t* bytes, int n, int flavor, PointG1* out, int32_t* codes) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint8_t* m = bytes + (size_t)i * 64;
  bool gx, gy;
  PointG1 P;
  fp_from_be(P.x, m, &gx);
  fp_from_be(P.y, m + 32, &gy);
  bool nz = false;
  for (int k = 0; k < 64; k++) nz |= m[k] != 0;
  int32_t code = HG_OK;
  P.inf = nz ? 0u : 1u;
  if (flavor == HG_FLAVOR_CF && (gx || gy)) {
    code = HG_ERR_CF_EXCEEDS;
  } else if (nz && !g1_on_curve(P.x, P.y)) {
    code = flavor == HG_FLAVOR_CF ? HG_ERR_CF_MALFORMED : HG_ERR_SIG_UNMARSHAL;
  }
  out[i] = P;
  codes[i] = code;
}

// ------------------------------------------------------------------ encode
__global__ void k_encode_g2(const PointG2* in, int n, uint8_t* out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t* o = out + (size_t)i * 128;
  PointG2 P = in[i];
  if (P.inf) {
    for (int k = 0; k < 128; k++) o[k] = 0;
    return;
  }
  fp_to_be(o, P.x.x);
  fp_to_be(o + 32, P.x.y);
  fp_to_be(o + 64, P.y.x);
  fp_to_be(o + 96, P.y.y);
}

__global__ void k_encode_g1(const PointG1* in, int n, uint8_t* out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t* o = out + (size_t)i * 64;
  PointG1 P = in[i];
  if (P.inf) {
    for (int k = 0; k < 64; k++) o[k] = 0;
    return;
  }
  fp_to_be(o, P.x);
  fp_to_be(o + 32, P.y);
}

// ------------------------------------------------------------------ scalar multiples
HG_DEV void be32_to_words(uint32_t* w, const uint8_t* b) {
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint8_t* q = b + (7 - i) * 4;
    w[i] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | q[3];
  }
}
// pk = k * G2 (G2.ScalarBaseMult)
__global__ void k_g2_mul_base(const uint8_t* scalars, int n, PointG2* out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t k[8];
  be32_to_words(k, scalars + (size_t)i * 32);
  G2J g, r;
  const Fp2 gx = HG_G2X, gy = HG_G2Y;
  g.x = gx;
  g.y = gy;
  f2_one(g.z);
  g2_mul(r, g, k);
  PointG2 P;
  if (g2_is_inf(r)) {
    f2_zero(P.x);
    f2_zero(P.y);
    P.inf = 1;
  } else {
    g2_affine(P.x, P.y, r);
    P.inf = 0;
  }
  out[i] = P;
}
// sig = k * H (G1.ScalarMult on the hashed message)
__global__ void k_g1_mul(const PointG1* base, const uint8_t* scalars, int n, PointG1* out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t k[8];
  be32_to_words(k, scalars + (size_t)i * 32);
  G1J g, r;
  g.x = base->x;
  g.y = base->y;
  fp_one(g.z);
  g1_mul(r, g, k);
  PointG1 P;
  if (g1_is_inf(r)) {
    fp_zero(P.x);
    fp_zero(P.y);
    P.inf = 1;
  } else {
    g1_affine(P.x, P.y, r);
    P.inf = 0;
  }
  out[i] = P;
}

// ------------------------------------------------------------------ hash-to-G1
// H = k * G1 where k is the hashedMessage scalar (validated on the host)
__global__ void k_hash_point(const uint32_t* k_words, PointG1* out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  G1J g;
  const Fp gx = HG_G1X, gy = HG_G1Y;
  g.x = gx;
  g.y = gy;
  fp_one(g.z);
  G1J h;
  g1_mul(h, g, k_words);
  PointG1 P;
  g1_affine(P.x, P.y, h);
  P.inf = 0;
  out[0] = P;
}

// ------------------------------------------------------------------ fixed G2Base lines
// Same step order as the Miller loop in k_verify: for i = 65..1 a doubling
// line, then an addition line when NAF[i-1] != 0, then the two Frobenius lines.
__global__ void k_g2_lines(LineCoef* tab) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const int8_t naf[kNafLen] = HG_NAF;
  const Fp2 qx = HG_G2X, qy = HG_G2Y;
  const Fp2 g1[6] = HG_GAMMA1;
  const Fp g2[6] = HG_GAMMA2;
  G2T R;
  R.x = qx;
  R.y = qy;
  f2_one(R.z);
  f2_one(R.t);
  Fp2 r2, nqy;
  f2_sqr(r2, qy);
  f2_neg(nqy, qy);
  int s = 0;
  for (int i = kNafLen - 1; i > 0; i--) {
    line_double(tab[s].a, tab[s].bx, tab[s].cy, R);
    s++;
    int d = naf[i - 1];
    if (d != 0) {
      line_add(tab[s].a, tab[s].bx, tab[s].cy, R, qx, d > 0 ? qy : nqy, r2);
      s++;
    }
  }
  Fp2 q1x, q1y, t;
  f2_conj(t, qx);
  f2_mul(q1x, t, g1[2]);
  f2_conj(t, qy);
  f2_mul(q1y, t, g1[3]);
  f2_sqr(r2, q1y);
  line_add(tab[s].a, tab[s].bx, tab[s].cy, R, q1x, q1y, r2);
  s++;
  Fp2 q2x;
  f2_muls(q2x, qx, g2[2]);
  f2_sqr(r2, qy);
  line_add(tab[s].a, tab[s].bx, tab[s].cy, R, q2x, qy, r2);
}

// ------------------------------------------------------------------ aggregation
// One 64-lane workgroup per request: lane l folds the registry points whose
// bit i has i % 64 == l with mixed additions, then an LDS tree reduction
// combines the 64 partial sums. The result is converted to affine by lane 0.
// Complement trick: when more than half the bits are set and a precomputed
// aligned block sum covers the request's range, sum = block - sum(unset).
__global__ __launch_bounds__(64) void k_aggregate(const PointG2* reg, int nreg, const AggRequest* reqs, int n,
                                                  const uint64_t* words, CheckIn* out, int32_t* codes) {
  __shared__ G2J part[64];
  int r = blockIdx.x;
  if (r >= n) return;
  AggRequest q = reqs[r];
  int lane = threadIdx.x;
  bool bad = (codes[r] != HG_OK);
  G2J acc;
  g2_set_inf(acc);
  uint32_t any = 0;
  if (!bad) {
    for (uint32_t i = lane; i < q.bitlen; i += 64) {
      uint64_t w = words[q.word_offset + (i >> 6)];
      if ((w >> (i & 63)) & 1) {
        any = 1;
        const PointG2& P = reg[q.offset + i];
        if (P.inf) continue;
        if (g2_is_inf(acc)) {
          acc.x = P.x;
          acc.y = P.y;
          f2_one(acc.z);
        } else {
          g2_add_affine(acc, acc, P.x, P.y);
        }
      }
    }
  }
  part[lane] = acc;
  uint64_t anyb = __ballot(any != 0);
  __syncthreads();
  for (int s = 32; s > 0; s >>= 1) {
    if (lane < s) {
      G2J o = part[lane + s];
      G2J m = part[lane];
      g2_add(m, m, o);
      part[lane] = m;
    }
    __syncthreads();
  }
  if (lane == 0) {
    CheckIn& C = out[r];
    if (bad) return;
    if (anyb == 0) {
      codes[r] = HG_ERR_EMPTY_AGG;
      C.pk.inf = 1;
      return;
    }
    G2J s = part[0];
    if (g2_is_inf(s)) {
      C.pk.inf = 1;
      f2_zero(C.pk.x);
      f2_zero(C.pk.y);
    } else {
      g2_affine(C.pk.x, C.pk.y, s);
      C.pk.inf = 0;
    }
  }
}

// ------------------------------------------------------------------ G1 combine
__global__ void k_g1_combine(const PointG1* a, const PointG1* b, int n, uint8_t* out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  G1J pa, pb, r;
  if (a[i].inf) g1_set_inf(pa); else { pa.x = a[i].x; pa.y = a[i].y; fp_one(pa.z); }
  if (b[i].inf) g1_set_inf(pb); else { pb.x = b[i].x; pb.y = b[i].y; fp_one(pb.z); }
  g1_add(r, pa, pb);
  uint8_t* o = out + (size_t)i * 64;
  if (g1_is_inf(r)) {
    for (int k = 0; k < 64; k++) o[k] = 0;
    return;
  }
  Fp x, y;
  g1_affine(x, y, r);
  fp_to_be(o, x);
  fp_to_be(o + 32, y);
}

// batched PublicKey.Combine (bn256/go/bn256.go:97-105): out[i] = a[i] + b[i] (G2)
__global__ void k_g2_combine(const PointG2* a, const PointG2* b, int n, PointG2* out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  G2J pa, pb, r;
  if (a[i].inf) g2_set_inf(pa); else { pa.x = a[i].x; pa.y = a[i].y; f2_one(pa.z); }
  if (b[i].inf) g2_set_inf(pb); else { pb.x = b[i].x; pb.y = b[i].y; f2_one(pb.z); }
  g2_add(r, pa, pb);
  PointG2 P;
  if (g2_is_inf(r)) {
    f2_zero(P.x);
    f2_zero(P.y);
    P.inf = 1;
  } else {
    g2_affine(P.x, P.y, r);
    P.inf = 0;
  }
  out[i] = P;
}

// ------------------------------------------------------------------ copy helpers
__global__ void k_checks_from_points(const PointG2* pks, const PointG1* sigs, int n, CheckIn* out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[i].pk = pks[i];
  out[i].sig = sigs[i];
}
__global__ void k_merge_codes(const int32_t* a, const int32_t* b, int n, int32_t* out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  // pk decode errors win over sig decode errors (the registry is decoded first)
  out[i] = a[i] != HG_OK ? a[i] : b[i];
}
__global__ void k_sig_into_checks(const PointG1* sigs, int n, CheckIn* out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[i].sig = sigs[i];
}
__global__ void k_extract_pk(const CheckIn* in, int n, PointG2* out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[i] = in[i].pk;
}

// ------------------------------------------------------------------ self test
// plain-integer words in -> Montgomery product -> plain-integer words out
__global__ void k_fp_mul(const uint32_t* a, const uint32_t* b, int n, uint32_t* out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Fp x, y, xm, ym, r, rp;
  words_to_limbs(x, a + 8 * i);
  words_to_limbs(y, b + 8 * i);
  fp_to_mont(xm, x);
  fp_to_mont(ym, y);
  fp_mul(r, xm, ym);
  fp_from_mont(rp, r);
  limbs_to_words(out + 8 * i, rp);
}

}  // namespace hg

// ------------------------------------------------------------------ launchers (C++ linkage)
namespace hg {
static inline int nblk(int n, int b) { return (n + b - 1) / b; }

void launch_decode_g2(const uint8_t* bytes, int n, int flavor, PointG2* out, int32_t* codes, hipStream_t s) {
  if (n > 0) k_decode_g2<<<nblk(n, 64), 64, 0, s>>>(bytes, n, flavor, out, codes);
}
void launch_decode_g1(const uint8_t* bytes, int n, int flavor, PointG1* out, int32_t* codes, hipStream_t s) {
  if (n > 0) k_decode_g1<<<nblk(n, 64), 64, 0, s>>>(bytes, n, flavor, out, codes);
}
void launch_encode_g2(const PointG2* in, int n, uint8_t* out, hipStream_t s) {
  if (n > 0) k_encode_g2<<<nblk(n, 64), 64, 0, s>>>(in, n, out);
}
void launch_encode_g1(const PointG1* in, int n, uint8_t* out, hipStream_t s) {
  if (n > 0) k_encode_g1<<<nblk(n, 64), 64, 0, s>>>(in, n, out);
}
void launch_g2_mul_base(const uint8_t* scalars, int n, PointG2* out, hipStream_t s) {
  if (n > 0) k_g2_mul_base<<<nblk(n, 64), 64, 0, s>>>(scalars, n, out);
}
void launch_g1_mul(const PointG1* base, const uint8_t* scalars, int n, PointG1* out, hipStream_t s) {
  if (n > 0) k_g1_mul<<<nblk(n, 64), 64, 0, s>>>(base, scalars, n, out);
}
void launch_hash_point(const uint32_t* k, PointG1* out, hipStream_t s) { k_hash_point<<<1, 64, 0, s>>>(k, out); }
void launch_g2_lines(LineCoef* tab, hipStream_t s) { k_g2_lines<<<1, 64, 0, s>>>(tab); }
void launch_aggregate(const PointG2* reg, int nreg, const AggRequest* reqs, int n, const uint64_t* words,
                      CheckIn* out, int32_t* codes, hipStream_t s) {
  if (n > 0) k_aggregate<<<n, 64, 0, s>>>(reg, nreg, reqs, n, words, out, codes);
}
void launch_g1_combine(const PointG1* a, const PointG1* b, int n, uint8_t* out, hipStream_t s) {
  if (n > 0) k_g1_combine<<<nblk(n, 64), 64, 0, s>>>(a, b, n, out);
}
void launch_checks_from_points(const PointG2* pks, const PointG1* sigs, int n, CheckIn* out, hipStream_t s) {
  if (n > 0) k_checks_from_points<<<nblk(n, 64), 64, 0, s>>>(pks, sigs, n, out);
}
void launch_merge_codes(const int32_t* a, const int32_t* b, int n, int32_t* out, hipStream_t s) {
  if (n > 0) k_merge_codes<<<nblk(n, 64), 64, 0, s>>>(a, b, n, out);
}
void launch_sig_into_checks(const PointG1* sigs, int n, CheckIn* out, hipStream_t s) {
  if (n > 0) k_sig_into_checks<<<nblk(n, 64), 64, 0, s>>>(sigs, n, out);
}
void launch_extract_pk(const CheckIn* in, int n, PointG2* out, hipStream_t s) {
  if (n > 0) k_extract_pk<<<nblk(n, 64), 64, 0, s>>>(in, n, out);
}
void launch_g2_combine(const PointG2* a, const PointG2* b, int n, PointG2* out, hipStream_t s) {
  if (n > 0) k_g2_combine<<<nblk(n, 64), 64, 0, s>>>(a, b, n, out);
}
void launch_fp_mul(const uint32_t* a, const uint32_t* b, int n, uint32_t* out, hipStream_t s) {
  if (n > 0) k_fp_mul<<<nblk(n, 64), 64, 0, s>>>(a, b, n, out);
}
}  // namespace hg
