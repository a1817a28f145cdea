// bn256_gt.hip — aggregate verification in GT (the default path of
// hg_verify_aggregate and its device / multisig variants).
//
// processing.go:342-368 verifies a multisignature as
//     e(H, sum of the level's set keys) == e(sig, G2Base)
// (bn256/go/bn256.go:82-94). H = hashedMessage(msg) is one point per Handel
// run and the keys come from a fixed registry, so by bilinearity
//     e(H, sum pk_i) = prod e(H, pk_i)
// and every factor can be computed ONCE per (message, registry): the engine
// keeps G_i = e(H, pk_i) and, as the G2 fold does for points, the products of
// every subset of every aligned 8-key window (256 GT values per window) and of
// every aligned power-of-two block. A request then costs
//   * a GT fold: one Fp12 product per nonzero window byte of its bitset (or
//     of the bitset's complement inside an aligned block: GT values are
//     unitary, so the complement's inverse is a conjugate — no inversion,
//     no affine conversion, nothing like k_agg_finish), and
//   * ONE Miller loop (G2Base at -sig, lines from the table) plus the final
//     exponentiation, compared with the folded value: the pk-side Miller loop
//     (G2 doubling and addition programs, the pk lines) is gone.
// The verdict is the reference's for every registry of keys in G2 (keys are
// k * G2Base; the same parity scope as k_verify).
//
// Team layouts: k_gt_keys / k_verify_sig use the pairing team region of
// k_verify (bn256_pairing.h); the fold kernels use the compact FOLD region of
// the generator (slots F, A, B, registers ZERO and ONE, pre-pass scratch:
// kFoldTeamElems elements: 9.6 KB per 4-team workgroup), so several fold
// waves share a SIMD, also beside k_verify_sig's waves.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "bn256_agg.h"
#include "bn256_decode.h"
#include "bn256_gt.h"
#include "bn256_pairing.h"
#include "bn256_sigfe.h"
#include "bn256_sigteam.h"

namespace hg {
static inline int nblk(int n, int b) { return (n + b - 1) / b; }

static constexpr int kFoldWords = kFoldTeamElems * 10;
static_assert(kFoldWords % 2 == 0, "8-byte aligned team regions");

// the FOLD region's constant registers (ZERO for padded products, ONE)
HG_DEV void fold_regs_init(const Team& T) {
  if (T.tl == 0) {
    Fp z, o;
    fp_zero(z);
    fp_one(o);
    st_fp_a8(T.base + (kFoldRegBase + 0) * 10, z.l);
    st_fp_a8(T.base + (kFoldRegBase + 1) * 10, o.l);
  }
  team_sync();
}
using IMulF = XInst<XP_MUL12F, S_A, S_A, S_B>;  // A = A * B in the FOLD region
// (the hint re-fetches the same round's words: measured 1-2 % faster for the
// fold than keeping them, which frees 10 VGPRs but not a wave per SIMD,
// profiles/r05fb_fold_refetch_ab.json)
HG_DEV void fold_mul(const Team& T, XStream& S) {
  team_sync();
  IMulF::run(T, S, xh<IMulF>());
}

// ------------------------------------------------------------------ per-(message, registry) tables
// G_i = e(H, pk_i): the pairing team programs of k_verify with the G2Base
// pairing switched off (unit lines), then the final exponentiation.
template <int TEAMS>
__global__ __launch_bounds__(64) void k_gt_keys(const PointG2* reg, int n, const LineCoef* tab, const PointG1* hpt,
                                                Gt* out) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[TEAMS * kTeamWords];
  Team T = make_team(lds, kTeamWords);
  uint32_t* F = team_regs(T);
  const int idx = blockIdx.x * TEAMS + (threadIdx.x >> 4);
  const bool valid = idx < n;
  const PointG2& Q = reg[valid ? idx : n - 1];
  CheckCtx C;
  C.qx = Q.x;
  C.qy = Q.y;
  C.hx = hpt->x;
  C.hy = hpt->y;
  C.sx = hpt->x;
  C.sy = hpt->y;
  C.use_q = Q.inf == 0;
  C.use_s = false;
  if (!C.use_q) {  // e(H, infinity) = 1: unit lines on a well-defined doubling chain
    const Fp2 gx = HG_G2X, gy = HG_G2Y;
    C.qx = gx;
    C.qy = gy;
  }
  XStream S = x_stream();
  team_miller_check(T, F, C, tab, false, S, final_exp_hint());
  team_final_exp_fc(T, F, S);  // the GT tables: FE^m (team_final_exp_fc)
  if (valid) gt_store(T, S_F, out + idx);
}

// Window subset products, first pass: for each window w and half h (keys
// 8w + 4h .. 8w + 4h + 3) the 16 products of the half's subsets, by the
// recurrence P(s) = P(s without its lowest bit) * G(lowest bit), kept in LDS;
// entries s (h = 0) and s << 4 (h = 1) of the window's table. Absent keys
// (past the registry) are 1.
__global__ __launch_bounds__(64) void k_gt_nib(const Gt* key, int nreg, int nwin, Gt* win) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[4 * kFoldWords];
  __shared__ __attribute__((aligned(16))) uint32_t dp[4][16 * kFp12Words];
  Team T = make_team(lds, kFoldWords);
  fold_regs_init(T);
  const int team = (threadIdx.x & 63) >> 4;
  const int task = blockIdx.x * 4 + team;
  const bool valid = task < 2 * nwin;
  const int w = valid ? task >> 1 : 0, h = task & 1;
  uint32_t* D = dp[team];
  XStream S = x_stream();
  Fp one;
  gt_one_value(one, T);
  if (T.active) st_fp_a8(D + T.e * 10, one.l);  // P(empty) = 1
#pragma unroll 1
  for (int s = 1; s < 16; s++) {
    const int lo = s & -s, rest = s ^ lo;
    if (rest == 0) {
      const int j = 31 - __clz(lo);
      const int kidx = 8 * w + 4 * h + j;
      gt_load_or_one(T, S_A, key + (kidx < nreg ? kidx : 0), kidx < nreg);
    } else {
      lds_fp12_copy(T, slot(T, S_A), D + rest * kFp12Words);
      lds_fp12_copy(T, slot(T, S_B), D + lo * kFp12Words);
      fold_mul(T, S);
    }
    team_sync();
    lds_fp12_copy(T, D + s * kFp12Words, slot(T, S_A));
  }
  team_sync();
  if (!valid) return;
  Gt* tw = win + (size_t)w * 256;
#pragma unroll 1
  for (int s = (h ? 1 : 0); s < 16; s++) {
    Fp v;
    ld_fp_a8(v, D + s * kFp12Words + T.e * 10);
    if (!T.active) continue;
    uint2* dst = (uint2*)__builtin_assume_aligned(tw[h ? s << 4 : s].w + 10 * T.e, 8);
#pragma unroll
    for (int i = 0; i < 5; i++) dst[i] = make_uint2(v.l[2 * i], v.l[2 * i + 1]);
  }
}

// Second pass: entry (hi << 4) | lo = entry(lo) * entry(hi << 4) for hi, lo
// != 0; one team per (window, hi), 15 products.
__global__ __launch_bounds__(64) void k_gt_cross(int nwin, Gt* win) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[4 * kFoldWords];
  Team T = make_team(lds, kFoldWords);
  fold_regs_init(T);
  const int task = blockIdx.x * 4 + ((threadIdx.x & 63) >> 4);
  const bool valid = task < 15 * nwin;
  const int w = valid ? task / 15 : 0, hi = valid ? task % 15 + 1 : 1;
  Gt* tw = win + (size_t)w * 256;
  XStream S = x_stream();
#pragma unroll 1
  for (int lo = 1; lo < 16; lo++) {
    gt_load(T, S_A, tw + lo);
    gt_load(T, S_B, tw + (hi << 4));
    fold_mul(T, S);
    team_sync();
    if (valid) gt_store(T, S_A, tw + ((hi << 4) | lo));
  }
}

// 16-key windows: entry (hi << 8) | lo = w8[2w][lo] * w8[2w + 1][hi]; one
// team per (window, hi), 256 products, the next left operand in flight.
__global__ __launch_bounds__(64) void k_gt_win16(const Gt* w8, int nwin8, int nwin16, Gt* w16) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[kTeams12 * kFoldWords];
  Team T = make_team12(lds, kFoldWords);  // five 12-lane teams per wave
  fold_regs_init(T);
  const int task = blockIdx.x * kTeams12 + team12_index();
  const bool valid = task < 256 * nwin16;
  const int w = valid ? task >> 8 : 0, hi = task & 255;
  const Gt* lo_tab = w8 + (size_t)(2 * w) * 256;
  const bool has_hi = 2 * w + 1 < nwin8;
  Gt* dst = w16 + (size_t)w * 65536 + (size_t)hi * 256;
  XStream S = x_stream();
  Fp hv, one, nxt;
  gt_one_value(one, T);
  gt_read(hv, w8 + (size_t)(has_hi ? 2 * w + 1 : 2 * w) * 256 + hi, T);
  fp_sel(hv, has_hi, hv, one);
  gt_read(nxt, lo_tab, T);
#pragma unroll 1
  for (int lo = 0; lo < 256; lo++) {
    gt_put(T, S_A, nxt, false);
    gt_put(T, S_B, hv, false);
    if (lo + 1 < 256) gt_read(nxt, lo_tab + lo + 1, T);
    fold_mul(T, S);
    team_sync();
    if (valid) gt_store(T, S_A, dst + lo);
  }
}


// Block products, one level: dst[j] = src[2j] * src[2j + 1] (the last block of
// a level may be clipped: src[2j + 1] absent -> 1). src entries `stride` apart.
__global__ __launch_bounds__(64) void k_gt_blocks(const Gt* src, int stride, int nsrc, Gt* dst, int ndst) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[4 * kFoldWords];
  Team T = make_team(lds, kFoldWords);
  fold_regs_init(T);
  const int j = blockIdx.x * 4 + ((threadIdx.x & 63) >> 4);
  const bool valid = j < ndst;
  const int a = valid ? 2 * j : 0;
  XStream S = x_stream();
  gt_load(T, S_A, src + (size_t)a * stride);
  gt_load_or_one(T, S_B, src + (size_t)(a + 1 < nsrc ? a + 1 : a) * stride, a + 1 < nsrc);
  fold_mul(T, S);
  team_sync();
  if (valid) gt_store(T, S_A, dst + j);
}

// ------------------------------------------------------------------ the fold of a batch
// Term encoding: bits 0..29 index a GT table, bit 30 = conjugate on load,
// bit 31 = the block table (else the window table).
static constexpr uint32_t kTermConj = 1u << 30, kTermBlk = 1u << 31, kTermIdx = kTermConj - 1;
HG_DEV const Gt* term_ptr(uint32_t t, const Gt* win, const Gt* blk) {
  return ((t & kTermBlk) ? blk : win) + (t & kTermIdx);
}

// Plan and terms (one wave per request). The pairing check compares with
//   Y = conj(agg) = prod conj(t)                 (plain fold: conj is a ring
//                                                  automorphism, so every term
//                                                  is loaded conjugated)
//   Y = conj(block * conj(prod)) = conj(block) * prod   (complemented fold:
//                                                  conj(block) is one more term)
// so a request is ONE product of m' = m + comp terms. Ranges in the batch's
// term and chunk lists are taken with atomics (their order is irrelevant);
// then the window-table index of every nonzero byte of the folded mask in
// registry-aligned windows, and the owner of each chunk. An empty bitset is
// the reference's nil-aggregate panic (HG_ERR_EMPTY_AGG).
#ifndef HG_PLAN_WAVES  // A/B knob: 4 measured slower (profiles/r05sk_small_kernels_ab.json)
#define HG_PLAN_WAVES 16
#endif
static constexpr int kPlanWaves = HG_PLAN_WAVES;  // requests per k_gt_plan workgroup (one wave each)
template <int W>
HG_DEV uint32_t nz_units(uint64_t x) {
  return W == 8 ? nz_bytes(x) : nz_halves(x);
}
// W: registry-aligned window width of the fold's table (8: the 256-entry
// tables, 16: the 65536-entry ones)
template <int W>
__global__ __launch_bounds__(64 * kPlanWaves) void k_gt_plan(const AggRequest* reqs, int n, const uint64_t* words,
                                                             int32_t* codes, int nreg, int levels, GtBlockIndex bi,
                                                             GtReq* plan, GtHdr* hdr, uint32_t* terms,
                                                             int2* ord, int cap, int chunk, int* multi) {
  constexpr uint32_t kUnits = 64 / W, kMask = (1u << W) - 1u, kShift = W == 8 ? 3 : 4;
  __shared__ int sm[kPlanWaves], sc[kPlanWaves], sb[kPlanWaves], sd[kPlanWaves], sl[kPlanWaves], ss[kPlanWaves];
  __shared__ int base_m, base_c, base_b, base_d, base_l, base_s;
  const int wv = threadIdx.x >> 6;
  const int r = blockIdx.x * kPlanWaves + wv;
  const int lane = threadIdx.x & 63;
  GtReq g;
  g.m = g.chunks = g.comp = g.k = g.term_off = g.chunk_off = 0;
  AggRequest q;
  q.offset = q.bitlen = q.level_size = q.word_offset = 0;
  bool go = r < n && codes[r] == HG_OK;
  if (go) {
    q = reqs[r];
    uint32_t cnt = 0, nzs = 0, nzu = 0;
    for (uint32_t wi = lane; wi < (q.bitlen + 63) / 64; wi += 64) cnt += __popcll(agg_word(q, words, wi));
    for (uint32_t v = lane; v < agg_nrwords_w<W>(q); v += 64) {
      nzs += nz_units<W>(agg_rword_w<W>(q, words, (int)v, false));
      nzu += nz_units<W>(agg_rword_w<W>(q, words, (int)v, true));
    }
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) {
      cnt += __shfl_xor(cnt, d);
      nzs += __shfl_xor(nzs, d);
      nzu += __shfl_xor(nzu, d);
    }
    const AggPlan p = agg_plan(q, cnt, nzs, nzu, nreg, levels);
    if (cnt == 0) {
      if (lane == 0) codes[r] = HG_ERR_EMPTY_AGG;
      go = false;
    } else {
      g.comp = p.comp ? 1 : 0;
      g.k = p.k;
      g.m = (int)p.m + g.comp;
      g.chunks = (g.m + chunk - 1) / chunk;
    }
  }
  // ranges in the batch's term and chunk lists, and places in k_gt_combine's
  // request lists (requests of more than 4 chunks first, so the combine's
  // longest requests start first, on SIMDs of their own): one atomic per
  // workgroup and list
  const bool big = g.chunks > 4, mid = g.chunks >= 2 && g.chunks <= 4;
  // k_gt_chunks' order: every chunk longer than half the chunk size first
  // (a request's full chunks and a long tail), the short tails last, so the
  // waves of the first resident round carry the long product chains
  const int tail = g.m % chunk;
  const int nshort = (tail > 0 && 2 * tail <= chunk) ? 1 : 0, nlong = g.chunks - nshort;
  if (lane == 0) {
    sm[wv] = g.m;
    sc[wv] = g.chunks;
    sb[wv] = big ? 1 : 0;
    sd[wv] = mid ? 1 : 0;
    sl[wv] = nlong;
    ss[wv] = nshort;
  }
  __syncthreads();
  if (threadIdx.x < 64) {  // wave 0: lanes i < kPlanWaves scan wave i's counts side by side
    const int i = threadIdx.x;
    const bool in = i < kPlanWaves;
    int v[6] = {in ? sm[i] : 0, in ? sc[i] : 0, in ? sb[i] : 0, in ? sd[i] : 0, in ? sl[i] : 0, in ? ss[i] : 0};
    int inc[6];
#pragma unroll
    for (int j = 0; j < 6; j++) inc[j] = v[j];
#pragma unroll
    for (int d = 1; d < kPlanWaves; d <<= 1) {
#pragma unroll
      for (int j = 0; j < 6; j++) {
        const int x = __shfl_up(inc[j], d);
        if (i >= d) inc[j] += x;
      }
    }
    int tot[6];
#pragma unroll
    for (int j = 0; j < 6; j++) tot[j] = __shfl(inc[j], kPlanWaves - 1);
    if (in) {
      sm[i] = inc[0] - v[0];
      sc[i] = inc[1] - v[1];
      sb[i] = inc[2] - v[2];
      sd[i] = inc[3] - v[3];
      sl[i] = inc[4] - v[4];
      ss[i] = inc[5] - v[5];
    }
    if (i == 0) {
      // three 64-bit atomics, issued together (no branch between them): the
      // counter pairs (terms, chunks), (big, mid), (nlong, nshort) are adjacent
      // ints (little-endian halves; no low half can carry into its high one)
      typedef unsigned long long u64;
      const u64 tc2 = atomicAdd(reinterpret_cast<u64*>(&hdr->terms), (u64)(unsigned)tot[0] | ((u64)(unsigned)tot[1] << 32));
      const u64 bd2 = atomicAdd(reinterpret_cast<u64*>(&hdr->big), (u64)(unsigned)tot[2] | ((u64)(unsigned)tot[3] << 32));
      const u64 ls2 = atomicAdd(reinterpret_cast<u64*>(&hdr->nlong), (u64)(unsigned)tot[4] | ((u64)(unsigned)tot[5] << 32));
      base_m = (int)(unsigned)tc2;
      base_c = (int)(tc2 >> 32);
      base_b = (int)(unsigned)bd2;
      base_d = (int)(bd2 >> 32);
      base_l = (int)(unsigned)ls2;
      base_s = (int)(ls2 >> 32);
    }
  }
  __syncthreads();
  g.term_off = base_m + sm[wv];
  g.chunk_off = base_c + sc[wv];
  if (r < n && lane == 0) plan[r] = g;
  if (lane == 0 && big) multi[base_b + sb[wv]] = r;
  if (lane == 0 && mid) multi[n + base_d + sd[wv]] = r;
  if (!go) return;  // no barrier below
  uint32_t at = g.term_off;
  if (g.comp) {
    if (lane == 0) {
      uint32_t t;
      if (g.k <= 3) {  // a block inside one 8-key window: that window's subset entry
        const uint32_t mask = ((1u << (1u << g.k)) - 1u) << (q.offset & (uint32_t)(W - 1));
        t = (q.offset >> kShift) * (kMask + 1u) + (mask & kMask);
      } else {
        t = kTermBlk | (uint32_t)(bi.base[g.k] + (q.offset >> g.k));
      }
      terms[at] = t | kTermConj;
    }
    at++;
  }
  const uint32_t nrw = agg_nrwords_w<W>(q);
  const uint32_t win0 = q.offset >> kShift;
  const uint32_t flag = g.comp ? 0u : kTermConj;
  for (uint32_t v0 = 0; v0 < nrw; v0 += 64) {
    const uint32_t v = v0 + lane;
    const uint64_t mb = v < nrw ? agg_rword_w<W>(q, words, (int)v, g.comp != 0) : 0;
    const uint32_t pc = nz_units<W>(mb);
    uint32_t inc = pc;  // inclusive prefix over the wave
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t x = __shfl_up(inc, d);
      if (lane >= d) inc += x;
    }
    uint32_t pos = at + inc - pc;
#pragma unroll
    for (uint32_t j = 0; j < kUnits; j++) {
      const uint32_t unit = (uint32_t)(mb >> (W * j)) & kMask;
      if (unit) terms[pos++] = ((win0 + kUnits * v + j) * (kMask + 1u) + unit) | flag;
    }
    at += __shfl(inc, 63);
  }
  const int lo = base_l + sl[wv];
  for (int c = lane; c < nlong; c += 64) ord[lo + c] = make_int2(g.chunk_off + c, r);
  if (nshort && lane == 0) ord[cap - 1 - (base_s + ss[wv])] = make_int2(g.chunk_off + g.chunks - 1, r);
}

// Chunks: each team multiplies the (at most `chunk`) terms of one chunk. A
// request of one chunk is finished here (its product is Y); the others leave
// partial products for k_gt_combine. A fixed grid walks the chunk list (the
// count is on the device); every wave runs to the same, wave-uniform bound.
// The next term is fetched from HBM into registers while the current product
// runs.
static_assert(kGtChunkTeams == kTeams12, "k_gt_chunks' teams per workgroup");
// minimum waves per SIMD the compiler sizes k_gt_chunks' registers for (A/B
// builds: 3 -> 168 VGPRs with 37 spills, fold alone 0.59 -> 0.66 ms,
// profiles/r05fa_fold_occupancy_ab.json; 1 = the compiler's choice, 200 VGPRs)
#ifndef HG_CHUNK_WAVES
#define HG_CHUNK_WAVES 1
#endif
__global__ __launch_bounds__(64, HG_CHUNK_WAVES) void k_gt_chunks(const Gt* win, const Gt* blk, const uint32_t* terms,
                                                  const int2* ord, int cap, const GtReq* plan, const GtHdr* hdr,
                                                  int chunk, Gt* partial, Gt* y) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[kTeams12 * kFoldWords];
  Team T = make_team12(lds, kFoldWords);  // five 12-lane teams per wave
  fold_regs_init(T);
  const int team = team12_index();
  const int total = hdr->chunks, nlong = hdr->nlong;
  XStream S = x_stream();
  for (int base = blockIdx.x * kTeams12; base < total; base += gridDim.x * kTeams12) {  // wave-uniform
    const int k = base + team;
    const bool valid = k < total && T.active;
    int first = 0, cnt = 0, r = 0, c = 0;
    bool single = false;
    if (valid) {
      const int2 e = k < nlong ? ord[k] : ord[cap - 1 - (k - nlong)];
      c = e.x;
      r = e.y;
      const GtReq g = plan[r];
      first = g.term_off + (c - g.chunk_off) * chunk;
      cnt = min(chunk, g.term_off + g.m - first);
      single = g.chunks == 1;
    }
    int maxc = cnt;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) maxc = max(maxc, __shfl_xor(maxc, d));
    // the chunk's term words, read once: lane tl of the team holds term tl
    // (terms past 12 are read from the list), so no table read waits on a
    // dependent index load
    const uint32_t my_t = T.tl < cnt ? terms[first + T.tl] : 0u;
    const int tbase = 12 * team;
    auto term = [&](int i) -> uint32_t {  // wave-uniform i: every lane runs the shuffle
      const uint32_t v = (uint32_t)__shfl((int)my_t, tbase + (i < 12 ? i : 0), 64);
      return i < 12 ? v : (i < cnt ? terms[first + i] : 0u);
    };
    Fp cur, n1, n2, one;
    gt_one_value(one, T);
    fp_zero(n1);
    fp_zero(n2);
    const uint32_t t0 = term(0);
    gt_read(cur, term_ptr(valid ? t0 : 0u, win, blk), T);
    fp_sel(cur, valid, cur, one);
    gt_put(T, S_A, cur, valid && (t0 & kTermConj) != 0);
    // two table values in flight across the products (a read of the 16-key
    // table is a fresh HBM page most of the time)
    uint32_t t1 = term(1), t2 = term(2);
    if (1 < cnt) gt_read(n1, term_ptr(t1, win, blk), T);
    if (2 < cnt) gt_read(n2, term_ptr(t2, win, blk), T);
#pragma unroll 1
    for (int i = 1; i < maxc; i++) {
      Fp v;
      fp_sel(v, i < cnt, n1, one);
      gt_put(T, S_B, v, i < cnt && (t1 & kTermConj) != 0);
      n1 = n2;
      t1 = t2;
      t2 = term(i + 2);
      if (i + 2 < cnt) gt_read(n2, term_ptr(t2, win, blk), T);
      fold_mul(T, S);
    }
    team_sync();
    if (valid) gt_store(T, S_A, single ? y + r : partial + c);
    team_sync();
  }
}

// Combine (one wave per request of two or more chunks): the 4 teams multiply
// every 4th partial, a 2-level tree joins them into Y.
// Workgroup b takes the b-th request of the big list, then of the mid list
// (k_gt_plan), so the requests with the longest chains are dispatched first.
__global__ __launch_bounds__(64) void k_gt_combine(int n, const GtHdr* hdr, const int* multi, const GtReq* plan,
                                                   const Gt* partial, Gt* y) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[4 * kFoldWords];
  const int b = blockIdx.x, nbig = hdr->big;
  if (b >= nbig + hdr->mid) return;  // one request per wave: uniform
  const int r = b < nbig ? multi[b] : multi[n + b - nbig];
  const GtReq g = plan[r];
  Team T = make_team(lds, kFoldWords);
  fold_regs_init(T);
  const int team = (threadIdx.x & 63) >> 4;
  XStream S = x_stream();
  const int rounds = (g.chunks + 3) / 4;
  gt_load_or_one(T, S_A, partial + (team < g.chunks ? g.chunk_off + team : 0), team < g.chunks);
  // the team's next partial in flight across the product
  Fp one, nx;
  gt_one_value(one, T);
  nx = one;
  int c = team + 4;
  if (c < g.chunks) gt_read(nx, partial + g.chunk_off + c, T);
#pragma unroll 1
  for (int i = 1; i < rounds; i++) {
    Fp v;
    fp_sel(v, c < g.chunks, nx, one);
    gt_put(T, S_B, v, false);
    c += 4;
    if (c < g.chunks) gt_read(nx, partial + g.chunk_off + c, T);
    fold_mul(T, S);
  }
  for (int d = 1; d < (g.chunks > 2 ? 4 : 2); d <<= 1) {
    team_sync();
    lds_fp12_copy(T, slot(T, S_B), lds + (team ^ d) * kFoldWords + S_A * kFp12Words);
    fold_mul(T, S);
  }
  team_sync();
  if (team == 0) gt_store(T, S_A, y + r);
}

// kStore: the signature is decoded here from its marshal (sig_bytes, the
// flavor's rules): the prologue that decodes it for the verdict codes runs on
// the side stream, off this kernel's critical path. A signature that fails to
// decode gives a meaningless FE value, which k_gt_compare never reads (its code
// is the decode error already).
// kPad: one pairing wave per SIMD (below); HG_SIG_PAD=0 launches the
// unpadded variant, two waves per SIMD when two batches are in flight
template <int TEAMS, bool kStore, bool kPad = (TEAMS == 4)>
__global__ __launch_bounds__(64) void k_verify_sig(const PointG1* sigs, const uint8_t* sig_bytes, int flavor, int n,
                                                   const LineCoef* tab, const Gt* y, Gt* fe, int32_t* codes) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[TEAMS * kSigTeamWords];
  // kStore runs beside the GT fold on another stream, whose waves share the
  // SIMDs: the pairing wave (the step's critical path) wins the issue
  // arbitration, the fold's waves take the cycles it leaves
  if (kStore) __builtin_amdgcn_s_setprio(3);
  // one pairing wave per SIMD: the kernel needs 233 VGPRs, which would let a
  // second batch's pairing waves (two contexts in flight) share SIMDs and
  // crowd the fold's workgroups out of the CU's LDS; marking v255 and one
  // AGPR used makes its allocation exceed half of the 512-entry file
  if constexpr (kPad) asm volatile("" ::: "v255", "a0");
  Team T = make_team(lds, kSigTeamWords);
  uint32_t* F = T.base + kSigRegBase * 10;
  const int idx = blockIdx.x * TEAMS + (threadIdx.x >> 4);
  const bool valid = idx < n;
  const int ci = valid ? idx : n - 1;
  PointG1 sg;
  if (kStore) (void)decode_g1_one(sig_bytes + (size_t)ci * 64, flavor, sg);
  else sg = sigs[ci];
  XStream S = x_stream();
  team_miller_sig(T, F, sg.x, sg.y, sg.inf == 0, tab, S, SigFE<SigProgs16>::final_exp_hint_s());
  SigFE<SigProgs16>::team_final_exp_fc_s(T, S);
  if (kStore) {
    team_sync();
    if (valid) gt_store(T, S_F, fe + idx);
    return;
  }
  gt_load(T, S_A, y + ci);
  team_sync();
  const bool ok = t12_equal(T, S_F, S_A);
  if (valid && T.tl == 0 && codes[idx] == HG_OK) codes[idx] = ok ? HG_OK : HG_ERR_SIG_INVALID;
}

// fe[r] == y[r] (both canonical: word equality) for every request still HG_OK;
// one wave per request, lane l < 60 compares words 2l, 2l + 1
__global__ __launch_bounds__(64) void k_gt_compare(const Gt* fe, const Gt* y, int n, int32_t* codes) {
  const int r = blockIdx.x;
  if (r >= n) return;
  const int l = threadIdx.x;
  bool eq = true;
  if (l < 60) {
    const uint2 a = reinterpret_cast<const uint2*>(fe[r].w)[l];
    const uint2 b = reinterpret_cast<const uint2*>(y[r].w)[l];
    eq = a.x == b.x && a.y == b.y;
  }
  const bool all = __ballot(!eq) == 0;
  if (l == 0 && codes[r] == HG_OK) codes[r] = all ? HG_OK : HG_ERR_SIG_INVALID;
}

// k_gt_compare plus the verdict bitset (hg_pack_verdicts_device's layout: bit
// j of byte b = request 8b + j valid), one wave per byte: the step's pack
// launch and its dependency gap fold into the comparison
__global__ __launch_bounds__(64) void k_gt_compare_bits(const Gt* fe, const Gt* y, int n, int32_t* codes,
                                                        uint8_t* bits) {
  const int b = blockIdx.x;
  const int l = threadIdx.x;
  uint2 a[8], v[8];
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const int r = min(8 * b + j, n - 1);
    a[j] = l < 60 ? reinterpret_cast<const uint2*>(fe[r].w)[l] : make_uint2(0, 0);
    v[j] = l < 60 ? reinterpret_cast<const uint2*>(y[r].w)[l] : make_uint2(0, 0);
  }
  bool mine = false;  // lane j: request 8b + j verified
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const bool all = __ballot(a[j].x != v[j].x || a[j].y != v[j].y) == 0;
    const int r = 8 * b + j;
    if (l == j && r < n) {
      int32_t c = codes[r];
      if (c == HG_OK) c = all ? HG_OK : HG_ERR_SIG_INVALID;
      codes[r] = c;
      mine = c == HG_OK;
    }
  }
  const uint64_t m = __ballot(mine);
  if (l == 0) bits[b] = (uint8_t)(m & 0xffu);
}

// ------------------------------------------------------------------ launchers
void launch_gt_keys(const PointG2* reg, int n, const LineCoef* tab, const PointG1* h, Gt* out, hipStream_t s) {
  if (n > 0) k_gt_keys<4><<<nblk(n, 4), 64, 0, s>>>(reg, n, tab, h, out);
}
void launch_gt_windows8(const Gt* key, int nreg, Gt* w8, int nwin8, hipStream_t s) {
  if (nwin8 <= 0) return;
  k_gt_nib<<<nblk(2 * nwin8, 4), 64, 0, s>>>(key, nreg, nwin8, w8);
  k_gt_cross<<<nblk(15 * nwin8, 4), 64, 0, s>>>(nwin8, w8);
}
void launch_gt_windows16(const Gt* w8, int nwin8, Gt* w16, int nwin16, hipStream_t s) {
  if (nwin16 <= 0) return;
  k_gt_win16<<<nblk(256 * nwin16, kTeams12), 64, 0, s>>>(w8, nwin8, nwin16, w16);
}
void launch_gt_blocks(const Gt* src, int stride, int nsrc, Gt* dst, int ndst, hipStream_t s) {
  if (ndst > 0) k_gt_blocks<<<nblk(ndst, 4), 64, 0, s>>>(src, stride, nsrc, dst, ndst);
}
void launch_gt_fold(const AggRequest* reqs, int n, const uint64_t* words, int32_t* codes, int nreg, int levels,
                    const Gt* win, const Gt* blk, const GtBlockIndex& bi, GtWork w, Gt* y, bool zero_hdr, hipStream_t s) {
  if (n <= 0) return;
  if (zero_hdr) (void)hipMemsetAsync(w.hdr, 0, sizeof(GtHdr), s);
  if (w.win_bits == 16)
    k_gt_plan<16><<<nblk(n, kPlanWaves), 64 * kPlanWaves, 0, s>>>(reqs, n, words, codes, nreg, levels, bi, w.plan,
                                                                  w.hdr, w.terms, w.ord, w.cap, w.chunk, w.multi);
  else
    k_gt_plan<8><<<nblk(n, kPlanWaves), 64 * kPlanWaves, 0, s>>>(reqs, n, words, codes, nreg, levels, bi, w.plan,
                                                                 w.hdr, w.terms, w.ord, w.cap, w.chunk, w.multi);
  k_gt_chunks<<<w.chunk_grid, 64, 0, s>>>(win, blk, w.terms, w.ord, w.cap, w.plan, w.hdr, w.chunk, w.partial, y);
  k_gt_combine<<<n, 64, 0, s>>>(n, w.hdr, w.multi, w.plan, w.partial, y);
}
void launch_verify_sig(const PointG1* sigs, int n, const LineCoef* tab, const Gt* y, int32_t* codes, hipStream_t s) {
  if (n > 0) k_verify_sig<4, false><<<nblk(n, 4), 64, 0, s>>>(sigs, nullptr, 0, n, tab, y, nullptr, codes);
}
// pad (the default): one pairing wave per SIMD (k_verify_sig above); lanes
// that keep two batches in flight launch the unpadded variant, so the second
// batch's waves share the SIMDs. Experiment knobs (A/B): HG_SIG_TEAMS=2 — two
// checks per wave, unpadded; HG_SIG_PAD=0/1 — overrides `pad`.
static int sig_env() {
  static const int v = [] {
    const char* t = getenv("HG_SIG_TEAMS");
    if (t && atoi(t) == 2) return 2;
    const char* p = getenv("HG_SIG_PAD");
    if (!p) return -1;
    return atoi(p) == 0 ? 0 : 1;
  }();
  return v;
}
// the two-wave teams for a padded launch of at most w2_max (<= kSigW2MaxN)
// checks; HG_SIG_W2=0 turns them off (A/B)
bool sig_w2_for(bool pad, int n, int w2_max) {
  static const bool on = [] {
    const char* e = getenv("HG_SIG_W2");
    return !e || atoi(e) != 0;
  }();
  return on && pad && n <= w2_max && n <= kSigW2MaxN;
}
int sig_w2_lane_max() {
  static const int v = [] {
    const char* e = getenv("HG_SIG_W2_LANE_MAX");
    return e ? atoi(e) : 0;
  }();
  return v;
}
void launch_sig_pairing(const uint8_t* sigs, int flavor, int n, const LineCoef* tab, Gt* fe, hipStream_t s,
                        bool pad, int w2_max) {
  if (n <= 0) return;
  const int env = sig_env();
  if (env < 0 && sig_w2_for(pad, n, w2_max)) {
    launch_sig_pairing_w2(sigs, flavor, n, tab, fe, s);
    return;
  }
  if (env == 2) {
    k_verify_sig<2, true><<<nblk(n, 2), 32, 0, s>>>(nullptr, sigs, flavor, n, tab, nullptr, fe, nullptr);
    return;
  }
  if (env >= 0) pad = env == 1;
  if (pad) k_verify_sig<4, true><<<nblk(n, 4), 64, 0, s>>>(nullptr, sigs, flavor, n, tab, nullptr, fe, nullptr);
  else k_verify_sig<4, true, false><<<nblk(n, 4), 64, 0, s>>>(nullptr, sigs, flavor, n, tab, nullptr, fe, nullptr);
}
void launch_gt_compare(const Gt* fe, const Gt* y, int n, int32_t* codes, hipStream_t s) {
  if (n > 0) k_gt_compare<<<n, 64, 0, s>>>(fe, y, n, codes);
}
void launch_gt_compare_bits(const Gt* fe, const Gt* y, int n, int32_t* codes, uint8_t* bits, hipStream_t s) {
  if (n > 0) k_gt_compare_bits<<<(n + 7) / 8, 64, 0, s>>>(fe, y, n, codes, bits);
}

}  // namespace hg
