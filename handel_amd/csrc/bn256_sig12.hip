// bn256_sig12.hip — the GT path's signature-side pairing on FIVE 12-lane teams
// per wave (k_verify_sig12), with the G2Base lines evaluated ahead
// (k_sig_lines).
//
// The check (processing.go:342-368 -> bn256/go/bn256.go:82-94, GT form in
// bn256_gt.hip) needs per signature FE(Miller(G2Base at -sig)). k_verify_sig
// runs it on 16-lane teams: lanes 0..11 own the twelve Fp coefficients of f,
// lanes 12..15 evaluate the next G2Base line at -sig beside f^2 — and idle
// through the final exponentiation, which is ~60 % of the kernel. Here the
// 85 line evaluations of every signature (b' = bx * x_sig, c' = cy * -y_sig:
// four Fp products per line, bn256_gt.hip team_miller_sig) run first, as
// their own wide kernel, into HBM; the pairing kernel then needs only lanes
// 0..11 of a team, and a wave carries five checks instead of four: 20 % fewer
// wave-instructions per batch for the same per-wave program (the team
// programs are the generator's 12-lane forms: every pre-pass value on lanes
// 0..11, tools/gen_g2_schedule.py PRE_LANES).
//
// Evaluated lines in HBM: ev[(s * n + c) * 4 + j], j = FB.x, FB.y, FC.x, FC.y
// of line s for check c (160 bytes; a wave's five teams read 800 contiguous
// bytes per line). 85 lines x 160 B = 13.6 KB per check. k_sig_scalars
// decodes each signature once, k_sig_lines runs one product per thread (n x
// 340 threads: the whole GPU, a few microseconds per batch).
//
// Team region (layout T, tools/gen_g2_schedule.py): five Fp12 slots and the
// register file, 92 elements (kSigTTeamElems; 94 before the shared-operand
// squaring of r06) — the final exponentiation parks two of its seven live
// values in HBM (bn256_sigfe.h team_final_exp_fc_t) — so a wave of five teams
// takes 18.4 KB of LDS and a CU holds eight pairing waves (two per SIMD: the
// unpadded kernels' 193-212 VGPRs allow it) beside a fold
// workgroup.
//
// Values are identical to k_verify_sig's (the same Montgomery products in the
// same order, canonical), so the FE values, and every verdict, are too.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "bn256_decode.h"
#include "bn256_g2sched.h"
#include "bn256_gt.h"
#include "bn256_sigfe.h"

namespace hg {

// threads per workgroup of the two small kernels ahead of the pairing (A/B
// knob: 64 measured slower, profiles/r05sk_small_kernels_ab.json)
#ifndef HG_SIG_LINE_BLOCK
#define HG_SIG_LINE_BLOCK 256
#endif
static constexpr int kLineBlock = HG_SIG_LINE_BLOCK;

// the signature's evaluation scalars: sc[2c] = x_sig, sc[2c + 1] = -y_sig
// (both 0 at infinity: e(inf, G2Base) = 1, every line evaluates to w^3, which
// the final exponentiation maps to 1 — bn256_gt.hip team_miller_sig). A
// signature that fails to decode gives meaningless lines: its FE value is
// never compared (its code is the decode error, k_agg_prologue).
__global__ __launch_bounds__(kLineBlock) void k_sig_scalars(const uint8_t* sig_bytes, int flavor, int n, Fp* sc) {
  const int c = blockIdx.x * kLineBlock + threadIdx.x;
  if (c >= n) return;
  PointG1 sg;
  (void)decode_g1_one(sig_bytes + (size_t)c * 64, flavor, sg);
  Fp nsy, z;
  fp_zero(z);
  fp_neg(nsy, sg.y);
  const bool use = sg.inf == 0;
  fp_sel(sc[2 * c], use, sg.x, z);
  fp_sel(sc[2 * c + 1], use, nsy, z);
}

// ev[(s * n + c) * 4 + j] = component j of line s at -sig_c: one Montgomery
// product per thread (FB = bx * x_sig, FC = cy * -y_sig); grid (4n / 256,
// lines), consecutive threads on consecutive 40-byte results
__global__ __launch_bounds__(kLineBlock) void k_sig_lines(const Fp* sc, int n, const LineCoef* tab, Fp* ev) {
  const int t = blockIdx.x * kLineBlock + threadIdx.x;  // 4 c + j
  if (t >= 4 * n) return;
  const int s = blockIdx.y;
  const int j = t & 3;
  const int c = t >> 2;
  const Fp a = reinterpret_cast<const Fp*>(&tab[s])[j];
  const Fp b = sc[2 * c + (j >> 1)];
  Fp o;
  fp_mul(o, a, b);
  uint2* dst = (uint2*)__builtin_assume_aligned(ev + (size_t)s * 4 * n + t, 8);
#pragma unroll
  for (int i = 0; i < 5; i++) dst[i] = make_uint2(o.l[2 * i], o.l[2 * i + 1]);
}

// The evaluated line reaches the team's registers FB, FC through one VGPR
// element per lane (lane tl < 4 holds Fp tl), read from HBM one publication
// ahead so the read's latency overlaps the rounds between.
struct EvPipe {
  Fp c;
};
HG_DEV void ev_fetch(const Team& T, EvPipe& P, const Fp* ev, int n, int ci, int s) {
  if (T.tl < 4) {
    const uint2* src = (const uint2*)__builtin_assume_aligned(ev + ((size_t)s * n + ci) * 4 + T.tl, 8);
#pragma unroll
    for (int i = 0; i < 5; i++) {
      const uint2 x = src[i];
      P.c.l[2 * i] = x.x;
      P.c.l[2 * i + 1] = x.y;
    }
  }
}
// the held line into FB, FC, then line `next` into flight
HG_DEV void ev_publish(const Team& T, uint32_t* F, EvPipe& P, const Fp* ev, int n, int ci, int next) {
  if (T.tl < 4) st_fp_a8(F + (R_FB_x + T.tl) * 10, P.c.l);
  team_sync();
  if (next < kNumLines) ev_fetch(T, P, ev, n, ci, next);
}

using ISqr12T = XInst<XP_SQR12_12_T, S_F, S_F>;
using ILineT = XInst<XP_LINE_FIX_12_T, S_F, S_F>;

// Miller(G2Base at -sig) over the NAF of 6u + 2 (bn256_gt.hip
// team_miller_sig's loop; the lines arrive evaluated): f^2, then f * line
// per digit (two lines on a nonzero digit), then the two Frobenius lines
HG_DEV void team_miller_sig12(const Team& T, uint32_t* F, const Fp* ev, int n, int ci, XStream& S, XHint after) {
  const int8_t naf[kNafLen] = HG_NAF;
  t12_set_one(T, S_F);
  if (T.tl == 0) {
    Fp zero, one;
    fp_zero(zero);
    fp_one(one);
    st_fp(F + R_ZERO * 10, zero);
    st_fp(F + R_ONE * 10, one);
  }
  team_sync();
  EvPipe P;
  fp_zero(P.c);
  ev_fetch(T, P, ev, n, ci, 0);
  int s = 0;
  for (int i = kNafLen - 1; i > 0; i--) {
    const int d = naf[i - 1];
    ev_publish(T, F, P, ev, n, ci, s + 1);  // line s, read by the product after f^2
    ISqr12T::run(T, S, xh<ILineT>());      // f^2 (f = 1 on the first digit)
    const XHint after_digit = i > 1 ? xh<ISqr12T>() : xh<ILineT>();
    if (d != 0) {
      ILineT::run(T, S, xh<ILineT>());
      ev_publish(T, F, P, ev, n, ci, s + 2);  // line s + 1 (the addition's)
      ILineT::run(T, S, after_digit);
      s += 2;
    } else {
      ILineT::run(T, S, after_digit);
      s += 1;
    }
  }
  // the two Frobenius lines
  ev_publish(T, F, P, ev, n, ci, s + 1);
  ILineT::run(T, S, xh<ILineT>());
  ev_publish(T, F, P, ev, n, ci, kNumLines);
  ILineT::run(T, S, after);
}

// fe[r] = FE(Miller(G2Base at -sig_r)) on layout T (kSigTTeamElems elements
// per team: 18.4 KB of LDS per wave), five teams per wave. The final
// exponentiation parks two values per check in HBM: fe[r] itself (the result
// overwrites it) and park[r]. kPad: one pairing wave per SIMD (as
// k_verify_sig's default); unpadded, two batches' waves share a SIMD.
template <bool kPad>
__global__ __launch_bounds__(64, kPad ? 1 : 2) void k_verify_sig12(const Fp* ev, int n, Gt* fe, Gt* park) {
  constexpr int kWords = kSigTTeamElems * 10;
  __shared__ __attribute__((aligned(16))) uint32_t lds[kTeams12 * kWords];
  // beside the GT fold on another stream: the pairing wave (the step's
  // critical path) wins the issue arbitration
  __builtin_amdgcn_s_setprio(3);
  if constexpr (kPad) asm volatile("" ::: "v255", "a0");
  Team T = make_team12(lds, kWords);
  uint32_t* F = T.base + kSigTRegBase * 10;
  const int idx = blockIdx.x * kTeams12 + team12_index();
  const bool valid = idx < n;
  const int ci = valid ? idx : n - 1;
  XStream S = x_stream();
  team_miller_sig12(T, F, ev, n, ci, S, SigFE<SigProgs12>::final_exp_hint_t());
  // parking records: res in fe[idx] (the result overwrites it), t0 in
  // park[idx]; a padding team (idx >= n) uses the spare records
  // park[n + 1 + (idx - n)] and park[n + 1 + kTeams12 + (idx - n)] (park has
  // n + 1 + 2 kTeams12 records, sig12_scalar_offset). Recomputed at each use.
  SigFE<SigProgs12>::team_final_exp_fc_t(T, S, [=](int k) -> uint32_t* {
    const int i = blockIdx.x * kTeams12 + team12_index();
    if (k == 0) return (i < n ? fe + i : park + n + 1 + (i - n))->w;
    return (i < n ? park + i : park + n + 1 + kTeams12 + (i - n))->w;
  });
  team_sync();
  Fp v;
  ld_fp_a8(v, slot(T, S_F) + T.e * 10);
  if (valid && T.active) {
    uint2* dst = (uint2*)__builtin_assume_aligned(fe[idx].w + 10 * T.e, 8);
#pragma unroll
    for (int i = 0; i < 5; i++) dst[i] = make_uint2(v.l[2 * i], v.l[2 * i + 1]);
  }
}

// ---------------------------------------------------------------- split form
// The same chain in three kernels, so that the one Fp inversion per check
// (the norm of f down to Fp, t12_inv_norm's Bernstein-Yang inversion: 4.3 %
// of k_verify_sig12's VALU instructions and 13 % of its SALU ones, measured
// by dropping it, profiles/r06p_inv_probe.json) is done for 256 checks at
// a time instead of once per wave:
//   k_sig12_miller  the Miller loop and the norm N = f conj(f) (bn256_sigfe.h
//                   fe_t_norm), then t12_inv_norm up to d (t12_inv_norm_terms):
//                   f -> fe[c], the terms -> hand[c], n = |d|^2 -> nrm[c]
//   k_sig12_ninv    nrm[c]^-1 for every check, by a product tree per 256
//                   checks and ONE inversion at its root
//   k_sig12_fe      f back into the team region, N^-1 from the terms and
//                   n^-1 (t12_inv_norm_finish), the rest of the chain
// The values are the monolithic kernel's, bit for bit: n^-1 is the unique
// canonical inverse either way, and every other operation is the same.
struct SigHand {
  Fp v[8];  // t0, t1, t2, d (x, y each)
};

// lane tl < 8 stores term value tl, lane 8 the norm (team-uniform values)
HG_DEV void sig12_store_terms(const Team& T, bool valid, const NormTerms& o, const Fp& nr, SigHand* hand, Fp* nrm) {
  if (valid && T.tl < 9) {
    Fp2 pick;  // (selects on values, not on member references: no scratch)
    f2_sel(pick, T.tl < 6, o.t2, o.d);
    f2_sel(pick, T.tl < 4, o.t1, pick);
    f2_sel(pick, T.tl < 2, o.t0, pick);
    Fp w;
    fp_sel(w, (T.tl & 1) == 0, pick.x, pick.y);
    fp_sel(w, T.tl == 8, nr, w);
    uint2* dst = (uint2*)__builtin_assume_aligned(T.tl == 8 ? nrm->l : hand->v[T.tl].l, 8);
#pragma unroll
    for (int i = 0; i < 5; i++) dst[i] = make_uint2(w.l[2 * i], w.l[2 * i + 1]);
  }
}

template <bool kPad>
__global__ __launch_bounds__(64, kPad ? 1 : 2) void k_sig12_miller(const Fp* ev, int n, Gt* fe, SigHand* hand,
                                                                   Fp* nrm) {
  constexpr int kWords = kSigTTeamElems * 10;
  __shared__ __attribute__((aligned(16))) uint32_t lds[kTeams12 * kWords];
  __builtin_amdgcn_s_setprio(3);
  if constexpr (kPad) asm volatile("" ::: "v255", "a0");
  Team T = make_team12(lds, kWords);
  uint32_t* F = T.base + kSigTRegBase * 10;
  const int idx = blockIdx.x * kTeams12 + team12_index();
  const bool valid = idx < n;
  const int ci = valid ? idx : n - 1;
  XStream S = x_stream();
  team_miller_sig12(T, F, ev, n, ci, S, xh<ISqr12T>());
  SigFE<SigProgs12>::fe_t_norm(T, S, xh_none());
  NormTerms o;
  Fp nr;
  t12_inv_norm_terms(T, S_B, o, nr);
  Fp v;
  ld_fp_a8(v, slot(T, S_F) + T.e * 10);
  if (valid && T.active) {
    uint2* dst = (uint2*)__builtin_assume_aligned(fe[idx].w + 10 * T.e, 8);
#pragma unroll
    for (int i = 0; i < 5; i++) dst[i] = make_uint2(v.l[2 * i], v.l[2 * i + 1]);
  }
  sig12_store_terms(T, valid, o, nr, hand + idx, nrm + idx);
}

// f = fe[c] into slot F of layout T, with the registers the programs read
HG_DEV void sig12_load_f(const Team& T, uint32_t* F, const Gt* fe, int ci) {
  if (T.tl == 0) {
    Fp zero, one;
    fp_zero(zero);
    fp_one(one);
    st_fp(F + R_ZERO * 10, zero);
    st_fp(F + R_ONE * 10, one);
  }
  const uint2* src = (const uint2*)__builtin_assume_aligned(fe[ci].w + 10 * T.e, 8);
  uint32_t v[10];
#pragma unroll
  for (int i = 0; i < 5; i++) {
    const uint2 x = src[i];
    v[2 * i] = x.x;
    v[2 * i + 1] = x.y;
  }
  if (T.active) st_fp_a8(slot(T, S_F) + T.e * 10, v);
  team_sync();
}

// k_sig12_miller's second half for a Miller value computed elsewhere (config
// 2's k_verify_ml, bn256_verify.hip): f = fe[c], the norm N = f conj(f)
// (fe_t_norm), then t12_inv_norm up to d: the terms -> hand[c], n -> nrm[c]
__global__ __launch_bounds__(64, 2) void k_sig12_norm(int n, const Gt* fe, SigHand* hand, Fp* nrm) {
  constexpr int kWords = kSigTTeamElems * 10;
  __shared__ __attribute__((aligned(16))) uint32_t lds[kTeams12 * kWords];
  __builtin_amdgcn_s_setprio(3);
  Team T = make_team12(lds, kWords);
  uint32_t* F = T.base + kSigTRegBase * 10;
  const int idx = blockIdx.x * kTeams12 + team12_index();
  const bool valid = idx < n;
  const int ci = valid ? idx : n - 1;
  XStream S = x_stream();
  sig12_load_f(T, F, fe, ci);
  SigFE<SigProgs12>::fe_t_norm(T, S, xh_none());
  NormTerms o;
  Fp nr;
  t12_inv_norm_terms(T, S_B, o, nr);
  sig12_store_terms(T, valid, o, nr, hand + idx, nrm + idx);
}

// ninv[c] = nrm[c]^-1 (0 for 0: never the case for a Miller value, whose
// lines all have the coefficient 1 at w^3, so f and its norms are nonzero;
// guarded so one value cannot spoil the other 255). Per block of 256 checks:
// a product tree in LDS (8 levels), one fp_inv at the root, the inverses
// back down (inv(left) = inv(parent) right, inv(right) = inv(parent) left).
static constexpr int kInvBlock = 256;
__global__ __launch_bounds__(kInvBlock) void k_sig12_ninv(const Fp* nrm, int n, Fp* ninv) {
  // levels of the tree: the 256 leaves at 0, then 128 nodes at 256, 64 at
  // 384, ..., the root at 510
  __shared__ Fp tree[2 * kInvBlock];
  const int t = threadIdx.x;
  const int c = blockIdx.x * kInvBlock + t;
  Fp x, one;
  fp_one(one);
  x = one;
  const bool use = c < n && !fp_is_zero(nrm[c]);
  if (use) x = nrm[c];
  tree[t] = x;
  __syncthreads();
  int off = 0;  // the level of 2 sz nodes being multiplied pairwise
  for (int sz = kInvBlock / 2; sz >= 1; sz >>= 1) {
    if (t < sz) fp_mul(tree[off + 2 * sz + t], tree[off + 2 * t], tree[off + 2 * t + 1]);
    off += 2 * sz;
    __syncthreads();
  }
  // off: the root's index
  if (t == 0) fp_inv(tree[off], tree[off]);
  __syncthreads();
  for (int sz = 1; sz <= kInvBlock / 2; sz <<= 1) {  // down: the 2 sz children of the level of sz nodes at off
    const int child = off - 2 * sz;
    Fp pinv, sib;
    if (t < 2 * sz) {
      pinv = tree[off + (t >> 1)];
      sib = tree[child + (t ^ 1)];
    }
    __syncthreads();
    if (t < 2 * sz) fp_mul(tree[child + t], pinv, sib);
    off = child;
    __syncthreads();
  }
  if (c < n) {
    Fp z;
    fp_zero(z);
    fp_sel(x, use, tree[t], z);
    ninv[c] = x;
  }
}

template <bool kPad>
__global__ __launch_bounds__(64, kPad ? 1 : 2) void k_sig12_fe(int n, Gt* fe, Gt* park, const SigHand* hand,
                                                               const Fp* ninv) {
  constexpr int kWords = kSigTTeamElems * 10;
  __shared__ __attribute__((aligned(16))) uint32_t lds[kTeams12 * kWords];
  __builtin_amdgcn_s_setprio(3);
  if constexpr (kPad) asm volatile("" ::: "v255", "a0");
  Team T = make_team12(lds, kWords);
  uint32_t* F = T.base + kSigTRegBase * 10;
  const int idx = blockIdx.x * kTeams12 + team12_index();
  const bool valid = idx < n;
  const int ci = valid ? idx : n - 1;
  XStream S = x_stream();
  sig12_load_f(T, F, fe, ci);  // the registers the programs read, f into slot F
  t12_conj(T, S_D, S_F);
  NormTerms o;
  const SigHand& h = hand[ci];
  o.t0.x = h.v[0];
  o.t0.y = h.v[1];
  o.t1.x = h.v[2];
  o.t1.y = h.v[3];
  o.t2.x = h.v[4];
  o.t2.y = h.v[5];
  o.d.x = h.v[6];
  o.d.y = h.v[7];
  t12_inv_norm_finish(T, S_B, o, ninv[ci]);
  // parking as k_verify_sig12
  SigFE<SigProgs12>::fe_t_rest(T, S, [=](int k) -> uint32_t* {
    const int i = blockIdx.x * kTeams12 + team12_index();
    if (k == 0) return (i < n ? fe + i : park + n + 1 + (i - n))->w;
    return (i < n ? park + i : park + n + 1 + kTeams12 + (i - n))->w;
  });
  team_sync();
  Fp v;
  ld_fp_a8(v, slot(T, S_F) + T.e * 10);
  if (valid && T.active) {
    uint2* dst = (uint2*)__builtin_assume_aligned(fe[idx].w + 10 * T.e, 8);
#pragma unroll
    for (int i = 0; i < 5; i++) dst[i] = make_uint2(v.l[2 * i], v.l[2 * i + 1]);
  }
}

bool sig12_for(bool pad, size_t n) {
  static const int mode = [] {
    const char* e = getenv("HG_SIG12");
    return e ? (atoi(e) != 0 ? 1 : 0) : -1;
  }();
  return n <= (size_t)kSig12MaxN && (mode == 1 || (mode == -1 && !pad));
}

// the split form (k_sig12_miller, k_sig12_ninv, k_sig12_fe) for unpadded
// launches unless HG_SIG12_SPLIT=0
static bool sig12_split() {
  static const bool on = [] {
    const char* e = getenv("HG_SIG12_SPLIT");
    return !e || atoi(e) != 0;
  }();
  return on;
}

// the evaluated lines, then (each 256-byte aligned) the parking records, the
// signatures' scalars, and the split form's hand-over records and norms
static size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }
static size_t sig12_park_offset(int n) { return align256((size_t)n * kNumLines * 4 * sizeof(Fp)); }
static size_t sig12_scalar_offset(int n) {
  return sig12_park_offset(n) + align256((size_t)(n + 1 + 2 * kTeams12) * sizeof(Gt));
}
static size_t sig12_hand_offset(int n) { return sig12_scalar_offset(n) + align256((size_t)n * 2 * sizeof(Fp)); }
static size_t sig12_norm_offset(int n) { return sig12_hand_offset(n) + align256((size_t)n * sizeof(SigHand)); }
static size_t sig12_ninv_offset(int n) { return sig12_norm_offset(n) + align256((size_t)n * sizeof(Fp)); }
size_t sig12_lines_bytes(int n) { return sig12_ninv_offset(n) + (size_t)n * sizeof(Fp); }

// The final exponentiation of n Miller values already in fe (config 2's
// k_verify_ml), in place: k_sig12_norm, k_sig12_ninv, k_sig12_fe. ws:
// fe12_ws_bytes(n) bytes (parking records, hand-over terms, norms, inverses).
static size_t fe12_hand_offset(int n) { return align256((size_t)(n + 1 + 2 * kTeams12) * sizeof(Gt)); }
static size_t fe12_norm_offset(int n) { return fe12_hand_offset(n) + align256((size_t)n * sizeof(SigHand)); }
static size_t fe12_ninv_offset(int n) { return fe12_norm_offset(n) + align256((size_t)n * sizeof(Fp)); }
size_t fe12_ws_bytes(int n) { return fe12_ninv_offset(n) + (size_t)n * sizeof(Fp); }
void launch_fe12(Gt* fe, int n, uint8_t* ws, hipStream_t s) {
  if (n <= 0 || n > kSig12MaxN) return;
  Gt* park = (Gt*)ws;
  SigHand* hand = (SigHand*)(ws + fe12_hand_offset(n));
  Fp* nrm = (Fp*)(ws + fe12_norm_offset(n));
  Fp* ninv = (Fp*)(ws + fe12_ninv_offset(n));
  const int blocks = (n + kTeams12 - 1) / kTeams12;
  k_sig12_norm<<<blocks, 64, 0, s>>>(n, fe, hand, nrm);
  k_sig12_ninv<<<(n + kInvBlock - 1) / kInvBlock, kInvBlock, 0, s>>>(nrm, n, ninv);
  k_sig12_fe<false><<<blocks, 64, 0, s>>>(n, fe, park, hand, ninv);
}

void launch_sig_pairing12(const uint8_t* sigs, int flavor, int n, const LineCoef* tab, Fp* ev, Gt* fe,
                          hipStream_t s, bool pad) {
  // k_sig_lines indexes 4 n threads in int (callers bound n by kSig12MaxN)
  if (n <= 0 || n > kSig12MaxN) return;
  uint8_t* base = (uint8_t*)ev;
  Gt* park = (Gt*)(base + sig12_park_offset(n));
  Fp* sc = (Fp*)(base + sig12_scalar_offset(n));
  k_sig_scalars<<<(n + kLineBlock - 1) / kLineBlock, kLineBlock, 0, s>>>(sigs, flavor, n, sc);
  k_sig_lines<<<dim3((4 * n + kLineBlock - 1) / kLineBlock, kNumLines), kLineBlock, 0, s>>>(sc, n, tab, ev);
  const int blocks = (n + kTeams12 - 1) / kTeams12;
  // the split form for unpadded launches only (batches in flight share the
  // SIMDs, so the inversion kernel's latency hides behind other batches'
  // waves); a padded launch runs alone at one wave per SIMD, where the single
  // kernel is faster (0.947 vs 0.964 ms per 4096, profiles/r06b_sig12_split_ab.json)
  if (sig12_split() && !pad) {
    SigHand* hand = (SigHand*)(base + sig12_hand_offset(n));
    Fp* nrm = (Fp*)(base + sig12_norm_offset(n));
    Fp* ninv = (Fp*)(base + sig12_ninv_offset(n));
    k_sig12_miller<false><<<blocks, 64, 0, s>>>(ev, n, fe, hand, nrm);
    k_sig12_ninv<<<(n + kInvBlock - 1) / kInvBlock, kInvBlock, 0, s>>>(nrm, n, ninv);
    k_sig12_fe<false><<<blocks, 64, 0, s>>>(n, fe, park, hand, ninv);
    return;
  }
  if (pad) k_verify_sig12<true><<<blocks, 64, 0, s>>>(ev, n, fe, park);
  else k_verify_sig12<false><<<blocks, 64, 0, s>>>(ev, n, fe, park);
}

}  // namespace hg
