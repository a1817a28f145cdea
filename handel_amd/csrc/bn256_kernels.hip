// bn256_kernels.hip — the HIP kernels of the BN256 BLS verification path.
//
//   k_decode_g2 / k_decode_g1   marshalled points -> affine Montgomery + codes
//                               (x/crypto / cloudflare Unmarshal rules, a9)
//   k_hash_point                k * G1 for the hashedMessage scalar (a7)
//   k_g2_lines                  the fixed G2Base line table (precomputed once)
//   k_verify                    product-of-pairings check, one 16-lane team
//                               per check: e(H, pk) * e(-sig, G2Base) == 1 (a6)
//   k_pair                      bn256.Pair(g1, g2) -> GT marshal (parity probe)
//   k_aggregate                 bitset-driven G2 Combine fold, one wave per
//                               request, LDS tree reduction (a3, a4, a5)
//   k_g1_combine                batched SigBLS.Combine (a8)
//   k_fp_mul                    field self-test
#include <hip/hip_runtime.h>

#include "bn256_kernels.h"
#include "bn256_g2team.h"

namespace hg {

// ------------------------------------------------------------------ diagnostics
// Built only with -DHG_DIAG (tools/diag.py builds a separate library): lane 0
// of every block accumulates s_memtime cycles per phase of k_verify.
#ifdef HG_DIAG
__shared__ uint64_t hg_diag_acc[16];
__device__ uint64_t g_diag[4096 * 16];
#define DIAG_T0() uint64_t diag_t0_ = __builtin_amdgcn_s_memtime()
#define DIAG_ADD(k)                                                     \
  do {                                                                  \
    uint64_t diag_t1_ = __builtin_amdgcn_s_memtime();                   \
    if (threadIdx.x == 0) hg_diag_acc[k] += diag_t1_ - diag_t0_;        \
    diag_t0_ = diag_t1_;                                                \
  } while (0)
#else
#define DIAG_T0() (void)0
#define DIAG_ADD(k) (void)0
#endif

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

// ------------------------------------------------------------------ team Miller loop + final exp
// LDS layout per team: 12 Fp12 slots followed by the per-check constants.
enum { S_F = 0, S_A, S_B, S_C, S_D, S_E, S_G, S_H, S_I, S_J, S_K, S_L, kSlots };
static constexpr int kTeamWords = kSlots * kFp12Words + kG2Regs * 10;
static constexpr int kTeamsPerBlock = 4;

// the pairing's final exponentiation (x/crypto optate.go finalExponentiation)
HG_DEV void team_final_exp(const Team& T, uint32_t* F) {
  DIAG_T0();
  t12_inv(T, S_A, S_F, S_K, S_L);  // A = f^-1
  DIAG_ADD(5);
  t12_conj(T, S_B, S_F);           // B = conj(f)
  t12_mul(T, S_F, S_B, S_A);       // t1 = f^(p^6 - 1)
  t12_frob2(T, S_A, S_F);
  t12_mul(T, S_F, S_F, S_A);       // t1 = t1^(p^2 + 1)
  t12_frob(T, S_A, S_F);           // fp
  t12_frob2(T, S_B, S_F);          // fp2
  t12_mul(T, S_A, S_A, S_B);
  t12_frob(T, S_B, S_B);           // fp3
  t12_mul(T, S_A, S_A, S_B);       // y0 = fp * fp2 * fp3
  DIAG_ADD(6);
  t12_pow_u_cyc(T, F, S_C, S_F);          // fu
  t12_pow_u_cyc(T, F, S_D, S_C);          // fu2
  t12_pow_u_cyc(T, F, S_E, S_D);          // fu3
  DIAG_ADD(7);
  t12_frob(T, S_G, S_C);
  t12_conj(T, S_G, S_G);           // y3 = conj(frob(fu))
  t12_frob(T, S_H, S_D);
  t12_mul(T, S_H, S_C, S_H);
  t12_conj(T, S_H, S_H);           // y4 = conj(fu * frob(fu2))
  t12_frob2(T, S_C, S_D);          // y2 = frob2(fu2)
  t12_conj(T, S_D, S_D);           // y5 = conj(fu2)
  t12_frob(T, S_I, S_E);
  t12_mul(T, S_I, S_E, S_I);
  t12_conj(T, S_I, S_I);           // y6 = conj(fu3 * frob(fu3))
  t12_cyc_sqr(T, F, S_K, S_I);
  t12_mul(T, S_K, S_K, S_H);
  t12_mul(T, S_K, S_K, S_D);       // t0 = y6^2 y4 y5
  t12_mul(T, S_J, S_G, S_D);
  t12_mul(T, S_J, S_J, S_K);       // t1 = y3 y5 t0
  t12_mul(T, S_K, S_K, S_C);       // t0 = t0 y2
  t12_cyc_sqr(T, F, S_J, S_J);
  t12_mul(T, S_J, S_J, S_K);
  t12_cyc_sqr(T, F, S_J, S_J);            // t1 = (t1^2 t0)^2
  t12_conj(T, S_L, S_F);           // y1 = conj(t1_easy)
  t12_mul(T, S_K, S_J, S_L);       // t0 = t1 y1
  t12_mul(T, S_J, S_J, S_A);       // t1 = t1 y0
  t12_cyc_sqr(T, F, S_K, S_K);
  t12_mul(T, S_F, S_K, S_J);       // result
  DIAG_ADD(6);
}

// Per-check inputs of the team Miller loop.
struct CheckCtx {
  Fp2 qx, qy;   // affine pk (a dummy valid point when the pk is infinity)
  Fp hx, hy;    // H (affine)
  Fp sx, sy;    // sig (affine)
  bool use_q;   // pk contributes (not infinity)
  bool use_s;   // sig contributes (not infinity)
};

// Writes the team's G2 register file: point R = (Q, 1, 1), Q, -Qy, Qy^2, the
// Frobenius images q1 = pi(Q), -q2 = (Qx gamma2[2], Qy) (optate.go miller),
// the G1 points and constants.
HG_DEV void g2_regs_init(const Team& T, uint32_t* F, const CheckCtx& C) {
  const Fp2 g1[6] = HG_GAMMA1;
  const Fp g2[6] = HG_GAMMA2;
  Fp2 nqy, r2, q1x, q1y, q1r2, q2x, t, one2, zero2;
  f2_neg(nqy, C.qy);
  f2_sqr(r2, C.qy);
  f2_conj(t, C.qx);
  f2_mul(q1x, t, g1[2]);
  f2_conj(t, C.qy);
  f2_mul(q1y, t, g1[3]);
  f2_sqr(q1r2, q1y);
  f2_muls(q2x, C.qx, g2[2]);
  f2_one(one2);
  f2_zero(zero2);
  Fp zero, one, nsy;
  fp_zero(zero);
  fp_one(one);
  fp_neg(nsy, C.sy);
  if (T.tl == 0) {
    auto put2 = [&](int rx, const Fp2& v) {
      st_fp(F + rx * 10, v.x);
      st_fp(F + (rx + 1) * 10, v.y);
    };
    st_fp(F + R_ZERO * 10, zero);
    st_fp(F + R_ONE * 10, one);
    st_fp(F + R_PX * 10, C.hx);
    st_fp(F + R_PY * 10, C.hy);
    st_fp(F + R_SX * 10, C.sx);
    st_fp(F + R_NSY * 10, nsy);
    put2(R_X_x, C.qx);
    put2(R_Y_x, C.qy);
    put2(R_Z_x, one2);
    put2(R_T_x, one2);
    put2(R_QX_x, C.qx);
    put2(R_QY_x, C.qy);
    put2(R_NQY_x, nqy);
    put2(R_R2_x, r2);
    put2(R_P1X_x, q1x);
    put2(R_P1Y_x, q1y);
    put2(R_P1R2_x, q1r2);
    put2(R_P2X_x, q2x);
    put2(R_F2ONE_x, one2);
    put2(R_F2ZERO_x, zero2);
  }
  team_sync();
}

// Loads the G2Base line s (a, bx, cy: 6 Fp) into FA, FBX, FCY.
HG_DEV void load_fixed_line(const Team& T, uint32_t* F, const LineCoef* tab, int s) {
  const Fp* src = reinterpret_cast<const Fp*>(&tab[s]);
  if (T.tl < 6) st_fp(F + (R_FA_x + T.tl) * 10, src[T.tl]);
  team_sync();
}

// f *= pk line (LA, LB, LC) and, when has_fixed, the G2Base line (FA, FB, FC).
// A point at infinity contributes the unit line (a = b = 0, c = 1); the choice
// is an address select, so teams of one wave stay convergent.
HG_DEV void apply_lines(const Team& T, const uint32_t* F, const CheckCtx& C, bool has_fixed) {
  t12_mul_line_regs(T, S_F, S_F, F, C.use_q ? R_LA_x : R_F2ZERO_x, C.use_q ? R_LB_x : R_F2ZERO_x,
                    C.use_q ? R_LC_x : R_F2ONE_x);
  if (has_fixed)
    t12_mul_line_regs(T, S_F, S_F, F, C.use_s ? R_FA_x : R_F2ZERO_x, C.use_s ? R_FB_x : R_F2ZERO_x,
                      C.use_s ? R_FC_x : R_F2ONE_x);
}

// f = Miller(pk at H) * Miller(G2Base at -sig) (x/crypto optate.go miller, with
// the two loops sharing their squarings); the G2 steps run as team programs.
HG_DEV void team_miller_check(const Team& T, uint32_t* F, const CheckCtx& C, const LineCoef* tab, bool has_fixed) {
  const int8_t naf[kNafLen] = HG_NAF;
  t12_set_one(T, S_F);
  g2_regs_init(T, F, C);
  int s = 0;
  DIAG_T0();
  for (int i = kNafLen - 1; i > 0; i--) {
    load_fixed_line(T, F, tab, s++);
    DIAG_ADD(0);
    g2_program(T, F, kProgDBL);
    DIAG_ADD(1);
    if (i != kNafLen - 1) t12_sqr_fast(T, F, S_F, S_F);
    DIAG_ADD(2);
    apply_lines(T, F, C, has_fixed);
    DIAG_ADD(3);
    int d = naf[i - 1];
    if (d != 0) {
      load_fixed_line(T, F, tab, s++);
      DIAG_ADD(0);
      if (d > 0) g2_program(T, F, kProgADD_POS);
      else g2_program(T, F, kProgADD_NEG);
      DIAG_ADD(4);
      apply_lines(T, F, C, has_fixed);
      DIAG_ADD(3);
    }
  }
  load_fixed_line(T, F, tab, s++);
  g2_program(T, F, kProgADD_F1);
  apply_lines(T, F, C, has_fixed);
  load_fixed_line(T, F, tab, s++);
  g2_program(T, F, kProgADD_F2);
  apply_lines(T, F, C, has_fixed);
}

HG_DEV uint32_t* team_regs(const Team& T) { return T.base + kSlots * kFp12Words; }

__global__ __launch_bounds__(64) void k_verify(const CheckIn* in, int n, const LineCoef* tab,
                                               const PointG1* hpt, int32_t* codes) {
  __shared__ uint32_t lds[kTeamsPerBlock * kTeamWords];
  Team T = make_team(lds, kTeamWords);
  uint32_t* F = team_regs(T);
  int idx = blockIdx.x * kTeamsPerBlock + (threadIdx.x >> 4);
  bool valid = idx < n;
  int ci = valid ? idx : n - 1;
  const CheckIn& I = in[ci];
  CheckCtx C;
  C.qx = I.pk.x;
  C.qy = I.pk.y;
  C.hx = hpt->x;
  C.hy = hpt->y;
  C.sx = I.sig.x;
  C.sy = I.sig.y;
  C.use_q = I.pk.inf == 0;
  C.use_s = I.sig.inf == 0;
  if (!C.use_q) {  // keep the (unused) doubling chain well-defined
    const Fp2 gx = HG_G2X, gy = HG_G2Y;
    C.qx = gx;
    C.qy = gy;
  }
#ifdef HG_DIAG
  if (threadIdx.x < 16) hg_diag_acc[threadIdx.x] = 0;
  __syncthreads();
  uint64_t diag_start = __builtin_amdgcn_s_memtime();
#endif
  team_miller_check(T, F, C, tab, true);
#ifdef HG_DIAG
  uint64_t diag_mid = __builtin_amdgcn_s_memtime();
#endif
  team_final_exp(T, F);
  bool ok = t12_is_one(T, S_F);
  if (valid && T.tl == 0 && codes[idx] == HG_OK) codes[idx] = ok ? HG_OK : HG_ERR_SIG_INVALID;
#ifdef HG_DIAG
  uint64_t diag_end = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0 && blockIdx.x < 4096) {
    for (int k = 0; k < 8; k++) g_diag[blockIdx.x * 16 + k] = hg_diag_acc[k];
    g_diag[blockIdx.x * 16 + 8] = diag_mid - diag_start;
    g_diag[blockIdx.x * 16 + 9] = diag_end - diag_mid;
    g_diag[blockIdx.x * 16 + 10] = diag_end - diag_start;
  }
#endif
}

// bn256.Pair(g1, g2).Marshal() for n pairs (GT = 1 when either is infinity)
__global__ __launch_bounds__(64) void k_pair(const PointG1* g1s, const PointG2* g2s, int n, const LineCoef* tab,
                                             uint8_t* gt_out) {
  __shared__ uint32_t lds[kTeamsPerBlock * kTeamWords];
  Team T = make_team(lds, kTeamWords);
  uint32_t* F = team_regs(T);
  int idx = blockIdx.x * kTeamsPerBlock + (threadIdx.x >> 4);
  bool valid = idx < n;
  int ci = valid ? idx : n - 1;
  PointG1 P = g1s[ci];
  PointG2 Q = g2s[ci];
  CheckCtx C;
  C.use_q = (P.inf == 0) && (Q.inf == 0);
  C.use_s = false;
  if (!C.use_q) {
    const Fp2 gx = HG_G2X, gy = HG_G2Y;
    Q.x = gx;
    Q.y = gy;
    const Fp hx = HG_G1X, hy = HG_G1Y;
    P.x = hx;
    P.y = hy;
  }
  C.qx = Q.x;
  C.qy = Q.y;
  C.hx = P.x;
  C.hy = P.y;
  fp_zero(C.sx);
  fp_zero(C.sy);
  team_miller_check(T, F, C, tab, false);
  team_final_exp(T, F);  // f == 1 when either input is infinity, and 1^e == 1
  // GT.Marshal order: coefficients 5,3,1,4,2,0, each as (x, y)
  if (valid && T.active) {
    const int pos[6] = {5, 2, 4, 1, 3, 0};  // position of coefficient k in the marshal
    Fp v;
    ld_fp(v, slot(T, S_F) + T.e * 10);
    // comp 0 (x) first, comp 1 (y) second
    uint8_t* o = gt_out + (size_t)idx * 384 + pos[T.k] * 64 + (T.comp ? 32 : 0);
    fp_to_be(o, v);
  }
}

// Team Fp12 op probe (parity tests of the building blocks): inputs/outputs are
// 384-byte GT-marshal-ordered canonical elements.
//   op 0 a*b, 1 a^2 (merged products), 2 cyclotomic a^2, 3 a^p, 4 a^(p^2),
//   5 a^-1, 6 conj(a), 7 a^u (cyclotomic), 8 final exponentiation
__global__ __launch_bounds__(64) void k_fp12_op(int op, const uint8_t* a, const uint8_t* b, int n, uint8_t* out) {
  __shared__ uint32_t lds[kTeamsPerBlock * kTeamWords];
  Team T = make_team(lds, kTeamWords);
  uint32_t* F = T.base + kSlots * kFp12Words;
  int idx = blockIdx.x * kTeamsPerBlock + (threadIdx.x >> 4);
  bool valid = idx < n;
  int ci = valid ? idx : n - 1;
  const int pos[6] = {5, 2, 4, 1, 3, 0};
  if (T.active) {
    Fp v;
    bool ge;
    fp_from_be(v, a + (size_t)ci * 384 + pos[T.k] * 64 + (T.comp ? 32 : 0), &ge);
    st_fp(slot(T, S_A) + T.e * 10, v);
    fp_from_be(v, b + (size_t)ci * 384 + pos[T.k] * 64 + (T.comp ? 32 : 0), &ge);
    st_fp(slot(T, S_B) + T.e * 10, v);
  }
  team_sync();
  {
    Fp z, one;
    fp_zero(z);
    fp_one(one);
    if (T.tl == 0) {
      st_fp(F + R_ZERO * 10, z);
      st_fp(F + R_ONE * 10, one);
    }
    team_sync();
  }
  // op bits 8..: repetitions (timing of one building block: reps - 1 extra
  // applications feed the result back as the input)
  int reps = (op >> 8) > 0 ? (op >> 8) : 1;
  op &= 255;
  for (int r = 0; r < reps; r++) {
    if (r > 0) t12_copy(T, S_A, S_F);
    switch (op) {  // kernel-uniform
      case 0: t12_mul(T, S_F, S_A, S_B); break;
      case 1: t12_sqr_fast(T, S_F, S_A); break;
      case 2: t12_cyc_sqr(T, S_F, S_A); break;
      case 3: t12_frob(T, S_F, S_A); break;
      case 4: t12_frob2(T, S_F, S_A); break;
      case 5: t12_inv(T, S_F, S_A, S_K, S_L); break;
      case 6: t12_conj(T, S_F, S_A); break;
      case 7: t12_pow_u_cyc(T, F, S_F, S_A); break;
      case 8: t12_copy(T, S_F, S_A); team_final_exp(T, F); break;
      case 9: t12_sqr_table(T, F, S_F, S_A); break;
      case 10: t12_cyc_sqr_table(T, F, S_F, S_A); break;
      default: t12_copy(T, S_F, S_A); break;
    }
  }
  if (valid && T.active) {
    Fp v;
    ld_fp(v, slot(T, S_F) + T.e * 10);
    fp_to_be(out + (size_t)idx * 384 + pos[T.k] * 64 + (T.comp ? 32 : 0), v);
  }
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
void launch_verify(const CheckIn* in, int n, const LineCoef* tab, const PointG1* h, int32_t* codes, hipStream_t s) {
  if (n > 0) k_verify<<<nblk(n, kTeamsPerBlock), 64, 0, s>>>(in, n, tab, h, codes);
}
void launch_pair(const PointG1* g1s, const PointG2* g2s, int n, const LineCoef* tab, uint8_t* gt, hipStream_t s) {
  if (n > 0) k_pair<<<nblk(n, kTeamsPerBlock), 64, 0, s>>>(g1s, g2s, n, tab, gt);
}
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
void launch_fp12_op(int op, const uint8_t* a, const uint8_t* b, int n, uint8_t* out, hipStream_t s) {
  if (n > 0) k_fp12_op<<<nblk(n, kTeamsPerBlock), 64, 0, s>>>(op, a, b, n, out);
}
int diag_read(uint64_t* out, size_t n) {
#ifdef HG_DIAG
  if (n > 4096 * 16) n = 4096 * 16;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_diag), n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : 1;
#else
  (void)out;
  (void)n;
  return -1;
#endif
}
void launch_fp_mul(const uint32_t* a, const uint32_t* b, int n, uint32_t* out, hipStream_t s) {
  if (n > 0) k_fp_mul<<<nblk(n, 64), 64, 0, s>>>(a, b, n, out);
}
}  // namespace hg
