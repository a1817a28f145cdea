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
#include "bn256_agg.h"
#include "bn256_curve.h"
#include "bn256_decode.h"

namespace hg {


// ------------------------------------------------------------------ decode
// Unmarshal rules:
//   go (x/crypto): exact length checked by the host; coordinates taken mod p;
//                  all-zero => infinity; else must be on the curve.
//   cf (cloudflare): each coordinate must be < p; all-zero => infinity; on
//                  the curve; G2 additionally in the order-n subgroup.
// The field and curve checks alone (the cf subgroup check, a scalar
// multiplication by the group order, is left to the caller): decode_g2_one
// and, for the pairing checks, k_decode_checks + k_checks_g2_subgroup.
HG_DEV int32_t decode_g2_fields(const uint8_t* m, int flavor, PointG2& P) {
  bool ge[4];
  bool nz = false;  // some byte nonzero (all-zero = infinity)
  fp_from_be(P.x.x, m, &ge[0], &nz);
  fp_from_be(P.x.y, m + 32, &ge[1], &nz);
  fp_from_be(P.y.x, m + 64, &ge[2], &nz);
  fp_from_be(P.y.y, m + 96, &ge[3], &nz);
  int32_t code = HG_OK;
  P.inf = nz ? 0u : 1u;
  if (flavor == HG_FLAVOR_CF && (ge[0] || ge[1] || ge[2] || ge[3])) code = HG_ERR_CF_EXCEEDS;
  else if (nz && !g2_on_curve(P.x, P.y)) code = flavor == HG_FLAVOR_CF ? HG_ERR_CF_MALFORMED : HG_ERR_PK_UNMARSHAL;
  return code;
}

// n * P == inf for an affine point on the twist (cloudflare twistPoint.IsOnCurve
// multiplies by Order)
HG_DEV bool g2_in_subgroup(const PointG2& P) {
  const uint32_t order[8] = {HG_ORDER32};
  G2J a, r;
  a.x = P.x;
  a.y = P.y;
  f2_one(a.z);
  g2_mul(r, a, order);
  return g2_is_inf(r);
}

HG_DEV int32_t decode_g2_one(const uint8_t* m, int flavor, PointG2& P) {
  int32_t code = decode_g2_fields(m, flavor, P);
  if (code == HG_OK && flavor == HG_FLAVOR_CF && !P.inf && !g2_in_subgroup(P)) code = HG_ERR_CF_MALFORMED;
  return code;
}

__global__ __launch_bounds__(64) void k_decode_g2(const uint8_t* bytes, int n, int flavor, PointG2* out, int32_t* codes) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  PointG2 P;
  const int32_t code = decode_g2_one(bytes + (size_t)i * 128, flavor, P);
  out[i] = P;
  codes[i] = code;
}

// G2 membership of decoded registry keys: *count += 1 for every key with
// n * key != inf (on the twist but outside the order-n subgroup G2). x/crypto's
// G2.Unmarshal (bn256/go/bn256.go:113-120) accepts such keys; the GT path's
// bilinearity argument only holds on G2, so a registry holding one is served
// by the G2 fold + two-pairing check instead (hg_api.cpp gt_max_level).
__global__ __launch_bounds__(64) void k_g2_subgroup(const PointG2* reg, int n, int* count) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const PointG2 P = reg[i];
  if (!P.inf) {
    const uint32_t order[8] = {HG_ORDER32};
    G2J a, r;
    a.x = P.x;
    a.y = P.y;
    f2_one(a.z);
    g2_mul(r, a, order);
    if (!g2_is_inf(r)) atomicAdd(count, 1);
  }
}

__global__ __launch_bounds__(64) void k_decode_g1(const uint8_t* bytes, int n, int flavor, PointG1* out, int32_t* codes) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  PointG1 P;
  const int32_t code = decode_g1_one(bytes + (size_t)i * 64, flavor, P);
  out[i] = P;
  codes[i] = code;
}

// Everything an aggregate-verification batch needs before its fold, in one
// launch (the GT path): the level check of processing.go:350-352, the
// signature decode (SigBLS.UnmarshalBinary, a9) and the verdict precedence
// sig decode error > level error > (fold: empty aggregate) > pairing verdict;
// block 0 also zeroes `zero_words` words (the fold's range counters).
__global__ __launch_bounds__(64) void k_agg_prologue(const AggRequest* reqs, int n, uint32_t nreg, const uint8_t* sigs,
                                                     int flavor, PointG1* pts, int32_t* codes, int* zero,
                                                     int zero_words) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (blockIdx.x == 0 && (int)threadIdx.x < zero_words) zero[threadIdx.x] = 0;
  if (i >= n) return;
  PointG1 P;
  int32_t code = decode_g1_one(sigs + (size_t)i * 64, flavor, P);
  pts[i] = P;
  const AggRequest r = reqs[i];
  const bool level_ok = r.bitlen == r.level_size && (uint64_t)r.offset + r.bitlen <= nreg;
  if (code == HG_OK && !level_ok) code = HG_ERR_LEVEL;
  codes[i] = code;
}

// cf only, after k_decode_checks: a pk that passed the field and curve checks
// but lies outside the order-n subgroup is HG_ERR_CF_MALFORMED, ahead of any
// signature error (pk errors come first). Its own kernel so that the decode
// kernel stays small: the scalar multiplication needs ~415 VGPRs, a whole
// SIMD's file, which inside k_decode_checks made every decode wave (go flavor
// included) wait for a SIMD the pairing waves of other batches had left empty.
__global__ __launch_bounds__(64) void k_checks_g2_subgroup(const CheckIn* in, int n, int32_t* codes) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int32_t c = codes[i];
  if (c == HG_ERR_CF_EXCEEDS || c == HG_ERR_CF_MALFORMED) return;  // the pk's own error already
  const PointG2 P = in[i].pk;
  if (!P.inf && !g2_in_subgroup(P)) codes[i] = HG_ERR_CF_MALFORMED;
}

// The pairing-check inputs in one pass (hg_verify_batch*): 64 checks per
// 128-thread block, wave 0 decodes the pks and wave 1 the sigs (the two run
// side by side instead of one after the other), straight into CheckIn; pk
// errors before sig errors (the order PublicKey.UnmarshalBinary / SigBLS
// unmarshal surface them).
__global__ __launch_bounds__(128) void k_decode_checks(const uint8_t* pks, const uint8_t* sigs, int n, int flavor,
                                                      CheckIn* out, int32_t* codes) {
  __shared__ int32_t sig_code[64];
  const int l = threadIdx.x & 63;
  const int i = blockIdx.x * 64 + l;
  const bool pk_wave = threadIdx.x < 64;  // wave-uniform
  int32_t a = HG_OK;
  if (i < n) {
    if (pk_wave) {
      PointG2 Q;
      a = decode_g2_fields(pks + (size_t)i * 128, flavor, Q);  // cf subgroup: k_checks_g2_subgroup
      out[i].pk = Q;
    } else {
      PointG1 S;
      sig_code[l] = decode_g1_one(sigs + (size_t)i * 64, flavor, S);
      out[i].sig = S;
    }
  }
  __syncthreads();
  if (pk_wave && i < n) codes[i] = a != HG_OK ? a : sig_code[l];
}

// ------------------------------------------------------------------ encode
__global__ __launch_bounds__(64) void k_encode_g2(const PointG2* in, int n, uint8_t* out) {
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

__global__ __launch_bounds__(64) void k_encode_g1(const PointG1* in, int n, uint8_t* out) {
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
__global__ __launch_bounds__(64) void k_g2_mul_base(const uint8_t* scalars, int n, PointG2* out) {
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
__global__ __launch_bounds__(64) void k_g1_mul(const PointG1* base, const uint8_t* scalars, int n, PointG1* out) {
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
__global__ __launch_bounds__(64) void k_hash_point(const uint32_t* k_words, PointG1* out) {
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
// Each line is stored divided by its constant coefficient a (LineCoef): the
// line products then take 4 Fp products per lane instead of 6 (the w^3 term
// is a coefficient shift), and the Fp2 factors are removed by the final
// exponentiation. No G2Base line has a = 0 (tests/test_oracle.py).
// Thread 0 walks the Miller loop and leaves x/crypto's lines in LDS; then one
// thread per line divides by a (85 Fp2 inversions side by side instead of one
// after another: the setup kernel 5.0 -> ~1.3 ms).
struct RawLine {
  Fp2 a, bx, cy;
};
__global__ __launch_bounds__(128) void k_g2_lines(LineCoef* tab) {
  __shared__ RawLine raw[kNumLines];
  if (threadIdx.x == 0) {
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
      line_double(raw[s].a, raw[s].bx, raw[s].cy, R);
      s++;
      int d = naf[i - 1];
      if (d != 0) {
        line_add(raw[s].a, raw[s].bx, raw[s].cy, R, qx, d > 0 ? qy : nqy, r2);
        s++;
      }
    }
    Fp2 q1x, q1y, t;
    f2_conj(t, qx);
    f2_mul(q1x, t, g1[2]);
    f2_conj(t, qy);
    f2_mul(q1y, t, g1[3]);
    f2_sqr(r2, q1y);
    line_add(raw[s].a, raw[s].bx, raw[s].cy, R, q1x, q1y, r2);
    s++;
    Fp2 q2x;
    f2_muls(q2x, qx, g2[2]);
    f2_sqr(r2, qy);
    line_add(raw[s].a, raw[s].bx, raw[s].cy, R, q2x, qy, r2);
  }
  __syncthreads();
  const int j = threadIdx.x;
  if (j < kNumLines) {
    Fp2 ai;
    f2_inv(ai, raw[j].a);
    f2_mul(tab[j].bx, raw[j].bx, ai);
    f2_mul(tab[j].cy, raw[j].cy, ai);
  }
}

// ------------------------------------------------------------------ aggregation
// The aggregate key of a request is the group sum of the registry keys whose
// bit is set (processing.go:355-363 folds PublicKey.Combine over them; the
// affine result is the same for any summation order).
//
// Block sums: Handel's level ranges are aligned power-of-two registry blocks
// clipped at N (partitioner.go:133-178), so hg_registry_load precomputes the
// sum of every aligned block [j 2^k, min((j+1) 2^k, N)) (k_block_sums, one
// level per launch). When more than half of a block-aligned request's bits are
// set, the kernel folds the UNSET keys and returns block - fold.
//
// k_aggregate, one 64-lane workgroup per request:
//   1. popcount of the bitset (lane-strided words, LDS reduction) -> set count,
//      complement decision, m = number of keys to fold;
//   2. compaction of the folded positions into LDS (per-word prefix offsets), so
//      lanes fold consecutive entries with no divergence on unset bits;
//   3. L = pow2 ~ m/2 lanes fold ceil(m/L) keys each with mixed additions, then a
//      log2(L)-level LDS tree of full additions (few levels for small requests);
//   4. lane 0 applies the block complement and converts to affine.
struct AggPartial {
  G2J s;          // fold of the set (or, complemented, the unset) keys
  uint32_t cnt;   // set bits
  int comp, k;    // complement at block level k
};
struct BlockIndex {
  int base[24];  // level k block j at blocks[base[k] + j]; level 0 is the registry
  int levels;    // highest level with a table
};

__global__ __launch_bounds__(64) void k_block_sums(const PointG2* src, int nsrc, PointG2* dst, int ndst) {
  int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= ndst) return;
  const PointG2& a = src[2 * j];
  G2J s;
  if (a.inf) g2_set_inf(s);
  else { s.x = a.x; s.y = a.y; f2_one(s.z); }
  if (2 * j + 1 < nsrc && !src[2 * j + 1].inf) g2_add_affine(s, s, src[2 * j + 1].x, src[2 * j + 1].y);
  PointG2 o;
  o.pad[0] = o.pad[1] = o.pad[2] = 0;
  if (g2_is_inf(s)) {
    f2_zero(o.x);
    f2_zero(o.y);
    o.inf = 1;
  } else {
    g2_affine(o.x, o.y, s);
    o.inf = 0;
  }
  dst[j] = o;
}

// Byte-window subset sums (hg_registry_load): for every aligned 8-key window w
// of the registry and every subset s of its keys, wsum[256 w + s] = the sum of
// reg[8 w + j] over the bits j of s (slots past the registry are absent). The
// fold then adds ONE table point per nonzero byte of the bitset instead of one
// key per set bit: 256 points x 176 B per 8 keys (22.5 MB for N = 4000) of HBM
// traded for ~2.5x fewer additions on the aggregation's critical path.
__global__ __launch_bounds__(64) void k_window_sums(const PointG2* reg, int nreg, PointG2* wsum, int nwin) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nwin * 256) return;
  const int w = i >> 8, sub = i & 255;
  G2J acc;
  g2_set_inf(acc);
  for (int j = 0; j < 8; j++) {
    const int slot = 8 * w + j;
    if (!((sub >> j) & 1) || slot >= nreg || reg[slot].inf) continue;
    g2_madd(acc, acc, reg[slot].x, reg[slot].y);
  }
  PointG2 o;
  o.pad[0] = o.pad[1] = o.pad[2] = 0;
  if (g2_is_inf(acc)) {
    f2_zero(o.x);
    f2_zero(o.y);
    o.inf = 1;
  } else {
    g2_affine(o.x, o.y, acc);
    o.inf = 0;
  }
  wsum[i] = o;
}

static constexpr int kAggPosCap = 64 * 8;  // window entries staged per pass (one word per lane)

// Schedule (one 1024-thread block): the plan of every request, then a counting
// sort by (lanes L descending, keys to fold descending). k_aggregate packs
// 64 / L consecutive requests of one bucket into a wave, so small requests
// share a wave (their folds and log2 L-level trees run side by side) and the
// heaviest single-request waves start first.
struct AggSched {
  int task_start[8];  // first task of lane class c (L = 64 >> c), task_start[7] = total
  int req_start[8];   // first entry of class c in order[]
  int nreq[7];
};
// Plan of every request: counts, complement decision, lanes; and its sort
// key for k_agg_order.
static constexpr int kAggSub = 64;  // cost sub-buckets inside a lane class
// One wave per request: the lanes scan the bitset's words side by side (the
// loads coalesce and overlap instead of one thread's serial chain of them).
__global__ __launch_bounds__(64) void k_agg_plan(const AggRequest* reqs, int n, const uint64_t* words,
                                                 const int32_t* codes, int nreg, int levels, AggPlan* plans,
                                                 int* keys) {
  const int r = blockIdx.x;
  const int lane = threadIdx.x;
  if (r >= n) return;
  AggPlan p;
  if (codes[r] != HG_OK) {
    p.cnt = 0;
    p.m = 0;
    p.k = 0;
    p.lanes = 1;
    p.comp = false;
  } else {
    const AggRequest q = reqs[r];
    uint32_t cnt = 0, nzs = 0, nzu = 0;
    for (uint32_t wi = lane; wi < (q.bitlen + 63) / 64; wi += 64) cnt += __popcll(agg_word(q, words, wi));
    for (uint32_t v = lane; v < agg_nrwords(q); v += 64) {
      nzs += nz_bytes(agg_rword(q, words, (int)v, false));
      nzu += nz_bytes(agg_rword(q, words, (int)v, true));
    }
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) {
      cnt += __shfl_xor(cnt, d);
      nzs += __shfl_xor(nzs, d);
      nzu += __shfl_xor(nzu, d);
    }
    p = agg_plan(q, cnt, nzs, nzu, nreg, levels);
  }
  if (lane != 0) return;
  plans[r] = p;
  int lg = 0;
  while ((1 << lg) < p.lanes) lg++;
  const uint32_t per = (p.m + p.lanes - 1) / p.lanes;  // table points per lane
  keys[r] = (6 - lg) * kAggSub + (kAggSub - 1 - (int)(per < (uint32_t)(kAggSub - 1) ? per : kAggSub - 1));
}

__global__ __launch_bounds__(1024) void k_agg_order(int n, const int* keys, int* order, AggSched* sched) {
  __shared__ int hist[7 * kAggSub];
  __shared__ int start[7 * kAggSub];
  const int tid = threadIdx.x;
  for (int i = tid; i < 7 * kAggSub; i += blockDim.x) hist[i] = 0;
  __syncthreads();
  for (int r = tid; r < n; r += blockDim.x) atomicAdd(&hist[keys[r]], 1);
  __syncthreads();
  if (tid == 0) {
    int acc = 0, tasks = 0;
    for (int c = 0; c < 7; c++) {
      int nc = 0;
      sched->req_start[c] = acc;
      for (int b = c * kAggSub; b < (c + 1) * kAggSub; b++) {
        start[b] = acc;
        acc += hist[b];
        nc += hist[b];
      }
      sched->nreq[c] = nc;
      sched->task_start[c] = tasks;
      const int per_wave = 1 << c;  // requests per wave for L = 64 >> c
      tasks += (nc + per_wave - 1) / per_wave;
    }
    sched->req_start[7] = acc;
    sched->task_start[7] = tasks;
  }
  __syncthreads();
  for (int r = tid; r < n; r += blockDim.x) order[atomicAdd(&start[keys[r]], 1)] = r;
}

// Cooperative Jacobian addition for the fold's LDS tree: the two lanes of a
// pair (the survivor, side A, and its partner, side B) each load BOTH partials
// (P = own, Q = partner's) and run ONE instruction stream on different data,
// so the add-2007-bl formula of g2_add costs each lane 9 Fp2 products instead
// of 16 (the tree's log2(L) sequential additions are the fold's critical path):
//   phase 1: zz = P.z^2, u = Q.x zz, s = Q.y (P.z zz)
//            side A: (Z1Z1, U2, S2), side B: (Z2Z2, U1, S1); swap through LDS;
//   phase 2: I = (2H)^2, J = H I (both), then the same three products on
//            selected operands — A: V = U1 I, (2r)^2, 2r (V - X3);
//            B: S1 J, (Z1 + Z2)^2, ((Z1 + Z2)^2 - Z1Z1 - Z2Z2) H = Z3 —
//            and B hands (S1 J, Z3) to A. Same formulas and field operations
//            as g2_add, so the survivor's result equals g2_add(P, Q).
// xo / xp: this lane's and the partner's 6-Fp2 exchange slots. Infinity and
// H = 0 (doubling or P = -Q) take g2_add's branches on both lanes alike.
HG_DEV void f2_st(uint32_t* p, const Fp2& a) {  // p 8-byte aligned: 64-bit LDS stores
  uint64_t* q = (uint64_t*)__builtin_assume_aligned(p, 8);
#pragma unroll
  for (int i = 0; i < 5; i++) {
    q[i] = (uint64_t)a.x.l[2 * i] | ((uint64_t)a.x.l[2 * i + 1] << 32);
    q[5 + i] = (uint64_t)a.y.l[2 * i] | ((uint64_t)a.y.l[2 * i + 1] << 32);
  }
}
HG_DEV void f2_ld(Fp2& a, const uint32_t* p) {
  const uint64_t* q = (const uint64_t*)__builtin_assume_aligned(p, 8);
#pragma unroll
  for (int i = 0; i < 5; i++) {
    const uint64_t vx = q[i], vy = q[5 + i];
    a.x.l[2 * i] = (uint32_t)vx;
    a.x.l[2 * i + 1] = (uint32_t)(vx >> 32);
    a.y.l[2 * i] = (uint32_t)vy;
    a.y.l[2 * i + 1] = (uint32_t)(vy >> 32);
  }
}
HG_DEV void f2_pick(Fp2& r, bool c, const Fp2& a, const Fp2& b) { f2_sel(r, c, a, b); }
HG_DEV void g2_add_pair(G2J& r, const G2J& P, const G2J& Q, bool side_a, uint32_t* xo, const uint32_t* xp) {
  if (g2_is_inf(P)) {
    r = Q;
    return;
  }
  if (g2_is_inf(Q)) {
    r = P;
    return;
  }
  Fp2 zz, u, s, t;
  f2_sqr(zz, P.z);
  f2_mul(u, Q.x, zz);
  f2_mul(t, P.z, zz);
  f2_mul(s, Q.y, t);
  f2_st(xo, zz);
  f2_st(xo + 20, u);
  f2_st(xo + 40, s);
  __syncthreads();
  Fp2 zz2, u2, s2;
  f2_ld(zz2, xp);
  f2_ld(u2, xp + 20);
  f2_ld(s2, xp + 40);
  __syncthreads();
  Fp2 z1z1, z2z2, U1, U2, S1, S2;
  f2_pick(z1z1, side_a, zz, zz2);
  f2_pick(z2z2, side_a, zz2, zz);
  f2_pick(U2, side_a, u, u2);
  f2_pick(U1, side_a, u2, u);
  f2_pick(S2, side_a, s, s2);
  f2_pick(S1, side_a, s2, s);
  Fp2 h, rr;
  f2_sub(h, U2, U1);
  f2_sub(rr, S2, S1);
  if (f2_is_zero(h)) {
    if (f2_is_zero(rr)) g2_double(r, P);  // P == Q as points
    else g2_set_inf(r);
    return;
  }
  Fp2 i, j, m1, m2, m3, x3, y2, zs;
  f2_dbl(t, h);
  f2_sqr(i, t);
  f2_mul(j, h, i);
  f2_dbl(rr, rr);
  // A: V = U1 I; B: S1 J
  Fp2 o1, o2;
  f2_pick(o1, side_a, U1, S1);
  f2_pick(o2, side_a, i, j);
  f2_mul(m1, o1, o2);
  // A: (2r)^2; B: (Z1 + Z2)^2
  f2_add(zs, P.z, Q.z);
  f2_pick(o1, side_a, rr, zs);
  f2_sqr(m2, o1);
  // A: X3 = (2r)^2 - J - 2V, y2 = V - X3; B: y2 = (Z1 + Z2)^2 - Z1Z1 - Z2Z2
  f2_sub(x3, m2, j);
  f2_sub(x3, x3, m1);
  f2_sub(x3, x3, m1);
  Fp2 ya, yb;
  f2_sub(ya, m1, x3);
  f2_sub(yb, m2, z1z1);
  f2_sub(yb, yb, z2z2);
  f2_pick(y2, side_a, ya, yb);
  // A: 2r (V - X3); B: Z3
  f2_pick(o1, side_a, rr, h);
  f2_mul(m3, o1, y2);
  f2_st(xo, m1);
  f2_st(xo + 20, m3);
  __syncthreads();
  Fp2 s1j, z3;
  f2_ld(s1j, xp);
  f2_ld(z3, xp + 20);
  __syncthreads();
  f2_dbl(s1j, s1j);
  r.x = x3;
  f2_sub(r.y, m3, s1j);
  r.z = z3;
}

// One wave per task: 64 / L requests of the same lane count L, one group of L
// lanes each. Per group: compaction of the nonzero window bytes of the folded
// mask (one registry-aligned word = 8 windows per lane and pass, segmented
// prefix sums), ceil(m / L) mixed additions of window subset sums per lane,
// then a log2(L)-level LDS tree; the group root is the request's partial sum.
__global__ __launch_bounds__(64) void k_aggregate(const PointG2* wsum, const AggRequest* reqs,
                                                  const uint64_t* words, const int* order, const AggPlan* plans,
                                                  const AggSched* sched, AggPartial* partial) {
  __shared__ G2J part[64];
  __shared__ __attribute__((aligned(16))) uint32_t xch[64 * 60];  // g2_add_pair exchange slots
  __shared__ uint32_t pos[kAggPosCap];
  __shared__ uint32_t cnt_lds[64];
  __shared__ uint32_t nw_lds[64];
  const int t = blockIdx.x;
  if (t >= sched->task_start[7]) return;  // uniform: fewer tasks than requests
  int c = 0;
  while (c < 6 && t >= sched->task_start[c + 1]) c++;
  const int L = 64 >> c;
  const int lane = threadIdx.x;
  const int g = lane / L, l = lane % L, gbase = g * L;
  const int idx = (t - sched->task_start[c]) * (1 << c) + g;
  const bool has = idx < sched->nreq[c];
  const int r = has ? order[sched->req_start[c] + idx] : -1;
  AggRequest q;
  q.offset = q.bitlen = q.level_size = q.word_offset = 0;
  AggPlan pl;
  pl.cnt = pl.m = 0;
  pl.k = 0;
  pl.lanes = L;
  pl.comp = false;
  if (has) {
    q = reqs[r];
    pl = plans[r];
  }
  const bool active = has && pl.cnt > 0;  // level errors and empty bitsets fold nothing
  const uint32_t nrw = active ? agg_nrwords(q) : 0;
  const uint32_t win0 = q.offset >> 3;  // first window of the request
  nw_lds[lane] = nrw;
  __syncthreads();
  uint32_t maxw = 0;
  for (int i = 0; i < 64; i += L) maxw = nw_lds[i] > maxw ? nw_lds[i] : maxw;  // wave-uniform
  G2J acc;
  g2_set_inf(acc);
  for (uint32_t v0 = 0; v0 < maxw; v0 += L) {
    const uint32_t v = v0 + l;
    const uint64_t mb = v < nrw ? agg_rword(q, words, (int)v, pl.comp) : 0;
    const uint32_t pc = nz_bytes(mb);
    cnt_lds[lane] = pc;
    __syncthreads();
    for (int d = 1; d < L; d <<= 1) {  // inclusive prefix inside the group
      const uint32_t x = l >= d ? cnt_lds[lane - d] : 0;
      __syncthreads();
      cnt_lds[lane] += x;
      __syncthreads();
    }
    const uint32_t total = cnt_lds[gbase + L - 1];
    uint32_t at = gbase * 8 + cnt_lds[lane] - pc;  // group region: 8 entries per lane
#pragma unroll
    for (int j = 0; j < 8; j++) {
      const uint32_t byte = (uint32_t)(mb >> (8 * j)) & 255u;
      if (byte) pos[at++] = ((uint32_t)(l * 8 + j) << 8) | byte;
    }
    __syncthreads();
    for (uint32_t e = l; e < total; e += L) {
      const uint32_t ent = pos[gbase * 8 + e];
      const PointG2& P = wsum[(size_t)(win0 + v0 * 8 + (ent >> 8)) * 256 + (ent & 255u)];
      if (!P.inf) g2_madd(acc, acc, P.x, P.y);
    }
    __syncthreads();
  }
  part[lane] = acc;
  __syncthreads();
  for (int s2 = L / 2; s2 > 0; s2 >>= 1) {
    // pairs (l, l + s2) add cooperatively; the other lanes pair with
    // themselves and discard the result (one instruction stream per wave)
    const bool side_a = l < s2;
    const int partner = side_a ? lane + s2 : (l < 2 * s2 ? lane - s2 : lane);
    const G2J P = part[lane];
    const G2J Q = part[partner];
    G2J res;
    g2_add_pair(res, P, Q, side_a, xch + lane * 60, xch + partner * 60);
    __syncthreads();
    if (side_a) part[lane] = res;
    __syncthreads();
  }
  if (has && l == 0) {
    AggPartial& o = partial[r];
    o.s = part[lane];
    o.cnt = pl.cnt;
    o.comp = pl.comp ? 1 : 0;
    o.k = pl.k;
  }
}

// One thread per request: block - fold for complemented requests, affine
// conversion (Bernstein-Yang inversion), empty-aggregate code.
__global__ __launch_bounds__(64) void k_agg_finish(const PointG2* blocks, BlockIndex bi, const AggRequest* reqs, int n,
                             const AggPartial* partial, CheckIn* out, int32_t* codes) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n || codes[r] != HG_OK) return;
  const AggPartial& pa = partial[r];
  CheckIn& C = out[r];
  if (pa.cnt == 0) {
    codes[r] = HG_ERR_EMPTY_AGG;
    C.pk.inf = 1;
    return;
  }
  G2J S = pa.s;
  if (pa.comp) {
    const PointG2& B = blocks[bi.base[pa.k] + (reqs[r].offset >> pa.k)];
    G2J nf = S;
    f2_neg(nf.y, S.y);
    if (B.inf) S = nf;
    else g2_madd(S, nf, B.x, B.y);
  }
  if (g2_is_inf(S)) {
    C.pk.inf = 1;
    f2_zero(C.pk.x);
    f2_zero(C.pk.y);
  } else {
    g2_affine(C.pk.x, C.pk.y, S);
    C.pk.inf = 0;
  }
}

// ------------------------------------------------------------------ G1 combine
__global__ __launch_bounds__(64) void k_g1_combine(const PointG1* a, const PointG1* b, int n, uint8_t* out) {
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
__global__ __launch_bounds__(64) void k_g2_combine(const PointG2* a, const PointG2* b, int n, PointG2* out) {
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
__global__ __launch_bounds__(64) void k_checks_from_points(const PointG2* pks, const PointG1* sigs, int n, CheckIn* out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[i].pk = pks[i];
  out[i].sig = sigs[i];
}
__global__ __launch_bounds__(64) void k_merge_codes(const int32_t* a, const int32_t* b, int n, int32_t* out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  // pk decode errors win over sig decode errors (the registry is decoded first)
  out[i] = a[i] != HG_OK ? a[i] : b[i];
}
// Verdict bitset (the one buffer distributed.py gathers across GPUs): bit j of
// byte b = check 8b + j passed (code 0); one thread per byte, tail bits 0.
__global__ __launch_bounds__(64) void k_pack_verdicts(const int32_t* codes, int n, uint8_t* bits) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= (n + 7) / 8) return;
  uint32_t v = 0;
  const int base = 8 * b;
#pragma unroll
  for (int j = 0; j < 8; j++)
    if (base + j < n && codes[base + j] == HG_OK) v |= 1u << j;
  bits[b] = (uint8_t)v;
}
__global__ __launch_bounds__(64) void k_sig_into_checks(const PointG1* sigs, int n, CheckIn* out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[i].sig = sigs[i];
}
__global__ __launch_bounds__(64) void k_extract_pk(const CheckIn* in, int n, PointG2* out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[i] = in[i].pk;
}

// ------------------------------------------------------------------ self test
// plain-integer words in -> Montgomery product -> plain-integer words out
__global__ __launch_bounds__(64) void k_fp_mul(const uint32_t* a, const uint32_t* b, int n, uint32_t* out) {
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
void launch_g2_subgroup(const PointG2* reg, int n, int* count, hipStream_t s) {
  if (n > 0) k_g2_subgroup<<<(n + 63) / 64, 64, 0, s>>>(reg, n, count);
}
void launch_decode_g1(const uint8_t* bytes, int n, int flavor, PointG1* out, int32_t* codes, hipStream_t s) {
  if (n > 0) k_decode_g1<<<nblk(n, 64), 64, 0, s>>>(bytes, n, flavor, out, codes);
}
void launch_agg_prologue(const AggRequest* reqs, int n, uint32_t nreg, const uint8_t* sigs, int flavor, PointG1* pts,
                         int32_t* codes, int* zero, int zero_words, hipStream_t s) {
  if (n > 0) k_agg_prologue<<<nblk(n, 64), 64, 0, s>>>(reqs, n, nreg, sigs, flavor, pts, codes, zero, zero_words);
}
void launch_decode_checks(const uint8_t* pks, const uint8_t* sigs, int n, int flavor, CheckIn* out, int32_t* codes,
                          hipStream_t s) {
  if (n <= 0) return;
  k_decode_checks<<<nblk(n, 64), 128, 0, s>>>(pks, sigs, n, flavor, out, codes);
  if (flavor == HG_FLAVOR_CF) k_checks_g2_subgroup<<<nblk(n, 64), 64, 0, s>>>(out, n, codes);
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
void launch_g2_lines(LineCoef* tab, hipStream_t s) { k_g2_lines<<<1, 128, 0, s>>>(tab); }
void launch_aggregate(const PointG2* wsum, int nreg, const PointG2* blocks, const int* block_base, int levels,
                      const AggRequest* reqs, int n, const uint64_t* words, int* order, void* partial_ws,
                      CheckIn* out, int32_t* codes, hipStream_t s) {
  AggPartial* partial = (AggPartial*)partial_ws;
  BlockIndex bi;
  bi.levels = levels < 23 ? levels : 23;
  for (int k = 0; k < 24; k++) bi.base[k] = k <= bi.levels ? block_base[k] : 0;
  if (n <= 0) return;
  AggPlan* plans = (AggPlan*)((uint8_t*)partial_ws + (size_t)n * sizeof(AggPartial));
  int* keys = (int*)(plans + n);
  AggSched* sched = (AggSched*)(keys + n);
  k_agg_plan<<<n, 64, 0, s>>>(reqs, n, words, codes, nreg, bi.levels, plans, keys);
  k_agg_order<<<1, 1024, 0, s>>>(n, keys, order, sched);
  k_aggregate<<<n, 64, 0, s>>>(wsum, reqs, words, order, plans, sched, partial);
  k_agg_finish<<<nblk(n, 64), 64, 0, s>>>(blocks, bi, reqs, n, partial, out, codes);
}
size_t agg_partial_bytes() { return sizeof(AggPartial) + sizeof(AggPlan) + sizeof(int); }
size_t agg_fixed_bytes() { return sizeof(AggSched); }
void launch_window_sums(const PointG2* reg, int nreg, PointG2* wsum, int nwin, hipStream_t s) {
  if (nwin > 0) k_window_sums<<<nblk(nwin * 256, 64), 64, 0, s>>>(reg, nreg, wsum, nwin);
}
void launch_block_sums(const PointG2* src, int nsrc, PointG2* dst, int ndst, hipStream_t s) {
  if (ndst > 0) k_block_sums<<<nblk(ndst, 64), 64, 0, s>>>(src, nsrc, dst, ndst);
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
void launch_pack_verdicts(const int32_t* codes, int n, uint8_t* bits, hipStream_t s) {
  if (n > 0) k_pack_verdicts<<<nblk((n + 7) / 8, 64), 64, 0, s>>>(codes, n, bits);
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
