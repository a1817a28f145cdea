// bn256_xprog.h — executor for the generated two-phase team programs
// (tables: bn256_xtab.h, from tools/gen_g2_schedule.py).
//
// A round makes every lane of a 16-lane team compute one Fp element
//     dst = REDC( sum_p U_p * V_p  +  R * sum_l lin_l )
// where U_p, V_p are Fp elements read from the team's LDS and lin_l are small
// multiples of Fp elements (the "x 1" slots of a program, added into the high
// columns so that REDC returns them unchanged). Operands that are linear
// combinations of several elements are materialised once per team by a
// pre-pass (phase 1): each lane evaluates up to NV of the round's distinct
// combinations into a scratch area, so the product phase (phase 2) is pure
// v_mad_u64_u32 work on LDS operands — no per-limb selects, no coefficient
// multiplies, no carries.
//
// Pre-pass terms are k * x (k > 0) or k * (4p - x) (k < 0: "negated"), summed
// limb-wise without carries: (4p)'' below is 4p with limbs in [2^26, 2^27 + 2^26)
// (top limb (4p >> 234) - 1), so (4p)''_l - x_l >= 0 for every element x below
// 2p. Elements are canonical except the results of the lazy rounds (LZ: the
// cyclotomic squaring's, in [0, 2p); only team programs read them). The
// generator bounds every limb sum below 2^32, every 64-bit column below 2^64
// and the REDC result: below 2p for product-only rounds (acc_reduce: one
// conditional subtraction), below 31p with linear terms (acc_reduce_wide,
// or its lazy form: the quotient estimate alone, [0, 2p)).
//
// Every table is bound to one call site: operands are absolute positions in
// the team region (Fp12 slot s element e -> element 12 s + e, register r ->
// element 144 + r), so an address is one add.
#pragma once
#include <utility>

#include "bn256_team.h"

namespace hg {

struct Team;
// Table prefetch (software pipelining of the per-lane round tables): every
// round starts by issuing the load of the NEXT round's words, so the ~600-cycle
// L1/L2 latency of the table read overlaps the current round's arithmetic
// instead of stalling its start. The stream remembers which round's words it
// holds; a round whose words are not there (no or a wrong hint) fetches them
// itself, so hints only affect speed, never results.
struct XHint {
  int off, w;  // table offset and per-lane stride of the round to prefetch (off < 0: none)
};
struct XStream;
template <int NV, int NT, int NP, int NL, int W, int NP2, int NL2, int KP, int KL1, int KL2, int KS1, int KS2, int LZ,
          int EF, int FU>
HG_DEV void x_round(const Team& T, XStream& S, int off, XHint nxt);


}  // namespace hg

#include "bn256_xtab.h"

namespace hg {

static constexpr uint32_t kP2N[10] = {HG_P2N};

struct XStream {
  uint32_t w[kXFetchWords];
  int off;  // table offset the words belong to (-1: none)
};
HG_DEV void x_fetch(const Team& T, XStream& S, XHint h) {
  const uint32_t* src = kXTab + h.off + T.tl * h.w;
#pragma unroll
  for (int i = 0; i < kXFetchWords; i++) S.w[i] = src[i];
  S.off = h.off;
}
HG_DEV XStream x_stream() {
  XStream S;
  S.off = -1;
  return S;
}
template <class I>
HG_DEV constexpr XHint xh() {
  return XHint{I::kOff, I::kW};
}
HG_DEV constexpr XHint xh_none() { return XHint{-1, 0}; }

template <int... I, typename Fn>
HG_DEV void x_static_for(std::integer_sequence<int, I...>, Fn&& f) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename Fn>
HG_DEV void x_for(Fn&& f) {
  x_static_for(std::make_integer_sequence<int, N>{}, f);
}

// 16-bit table entries: operands and destinations are byte offsets into the
// team region (0xffff = none); a linear term is element index << 8 | (int8) coef.
template <int W>
HG_DEV uint32_t x_half(const uint32_t (&w)[W], int i) {
  return (i & 1) ? (w[i >> 1] >> 16) : (w[i >> 1] & 0xffffu);
}
template <int W>
HG_DEV uint32_t x_off(const uint32_t (&w)[W], int i) {
  return x_half(w, i);
}
template <int W>
HG_DEV uint32_t x_term_off(const uint32_t (&w)[W], int i) {
  return (x_half(w, i) >> 8) * 40u;
}
template <int W>
HG_DEV int32_t x_coef(const uint32_t (&w)[W], int i) {
  return (int32_t)(int8_t)(x_half(w, i) & 255u);
}
HG_DEV uint32_t* x_at(const Team& T, uint32_t byte_off) {
  return (uint32_t*)__builtin_assume_aligned((uint8_t*)T.base + byte_off, 8);
}

// Evaluates sum_t c_t * x_t + K (2p)'' into out[10] as 32-bit limbs, where K
// (a round constant from the generator) is at least the sum of |c_t| over the
// negative c_t of every lane's combination, so every limb is a non-negative
// exact sum: one 32-bit multiply-add per limb and term, the correction folded
// into constants.
// K < 0: the correction is each lane's own sum of negative coefficients (a
// runtime multiply), for rounds where a uniform K would overflow a bound.
template <int W, int NT, int K>
HG_DEV void x_lincomb(const Team& T, const uint32_t (&w)[W], int base, uint32_t (&out)[10]) {
  uint32_t acc[10];
#pragma unroll
  for (int l = 0; l < 10; l++) acc[l] = K >= 0 ? (uint32_t)K * kP2N[l] : 0u;
  uint32_t negk = 0;
  x_for<NT>([&](auto t) {
    const uint32_t off = x_term_off(w, base + t);
    const int32_t c = x_coef(w, base + t);
    Fp x;
    ld_fp_a8(x, x_at(T, off));
    if constexpr (K < 0) negk += c < 0 ? (uint32_t)-c : 0u;
#pragma unroll
    for (int l = 0; l < 10; l++) acc[l] += (uint32_t)c * x.l[l];
  });
#pragma unroll
  for (int l = 0; l < 10; l++) out[l] = K >= 0 ? acc[l] : acc[l] + negk * kP2N[l];
}

// x_lincomb on operands already loaded (xs[t] = the element of term t)
template <int W, int NT, int K>
HG_DEV void x_lincomb_sum(const uint32_t (&w)[W], int base, const Fp (&xs)[NT], uint32_t (&out)[10]) {
  uint32_t acc[10];
#pragma unroll
  for (int l = 0; l < 10; l++) acc[l] = K >= 0 ? (uint32_t)K * kP2N[l] : 0u;
  uint32_t negk = 0;
#pragma unroll
  for (int t = 0; t < NT; t++) {
    const int32_t c = x_coef(w, base + t);
    if constexpr (K < 0) negk += c < 0 ? (uint32_t)-c : 0u;
#pragma unroll
    for (int l = 0; l < 10; l++) acc[l] += (uint32_t)c * xs[t].l[l];
  }
#pragma unroll
  for (int l = 0; l < 10; l++) out[l] = K >= 0 ? acc[l] : acc[l] + negk * kP2N[l];
}

// One job: sum of NP products of LDS operands plus NL R-shifted linear terms,
// reduced once. Entries from `base`: NP x (u, v), NL x term, dst.
//
// Issue order matters more than instruction count here: with one wave per
// SIMD nothing hides the latency of a dependent v_mad_u64_u32, and left alone
// the scheduler hoists every operand load of the job to the top (24 x 10
// VGPRs for a 12-product job) and, out of registers, walks the product column
// by column through ONE accumulator — a serial chain of dependent mads. Each
// product therefore runs in its own scheduling region (operand-scanning order:
// the 100 mads of a product hit 19 different columns, so consecutive mads are
// independent), with the next product's operands loaded at the top of the
// region so the LDS latency overlaps the current product's mads.
// acc += x * y in operand-scanning order, each partial product ONE
// v_mad_u64_u32 into its column. The empty asm after each mad keeps LLVM from
// reassociating a column's terms into a fresh serial chain (sum the products
// of column k in a temporary, then add it to the accumulator), which is what
// it does otherwise; the columns then stay independent chains of NP mads.
HG_DEV void acc_mad_pinned(Acc& a, const Fp& x, const Fp& y) {
#pragma unroll
  for (int i = 0; i < 10; i++)
#pragma unroll
    for (int j = 0; j < 10; j++) {
      a.c[i + j] += (uint64_t)x.l[i] * y.l[j];
      asm("" : "+v"(a.c[i + j]));
    }
}
// REDC digits interleaved with the job's last product (acc_mad_redc) where the
// generator sets a round's FU flag (the pairing kernels' single-job rounds:
// one wave per SIMD has nothing else to hide the reduction's serial chain
// behind; the GT fold runs several waves per SIMD and keeps the
// products-then-REDC order). HG_REDC_FUSE=0 builds that order everywhere.
#ifndef HG_REDC_FUSE
#define HG_REDC_FUSE 1
#endif

// a, b: the first product's operands, already loaded by the caller.
// FUSE: the last product runs with REDC digits 0..9 (acc_mad_redc).
template <int W, int NP, bool FUSE>
HG_DEV void x_products(const Team& T, const uint32_t (&w)[W], int base, Acc& acc, Fp a, Fp b) {
  if constexpr (NP > 0) {
    x_for<NP>([&](auto p) {
      Fp a2, b2;
      if constexpr (p + 1 < NP) {
        ld_fp_a8(a2, x_at(T, x_off(w, base + 2 * (p + 1))));
        ld_fp_a8(b2, x_at(T, x_off(w, base + 2 * (p + 1) + 1)));
      }
      if constexpr (FUSE && p + 1 == NP) acc_mad_redc(acc, a, b);
      else acc_mad_pinned(acc, a, b);
      // pin the columns here: the mads of product p stay in this region
      // (and are not sunk past the store's branch with the rest of the job)
#pragma unroll
      for (int c = 0; c < 21; c++) asm volatile("" : "+v"(acc.c[c]));
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (p + 1 < NP) {
        a = a2;
        b = b2;
      }
    });
  }
}
// Karatsuba products (the generator's per-job flag KS: jobs of 4+ products,
// where the combination's ~55 instructions are repaid): with x = x0 +
// 2^130 x1, y = y0 + 2^130 y1 (5-limb halves), a product is x0 y0, x1 y1 and
// (x0 + x1)(y0 + y1) - x0 y0 - x1 y1: 75 mads instead of 100, plus 10 limb
// additions. The three half-products accumulate over the whole job in their
// own 9-column sets and combine into the job's columns once. Every column sum
// and difference is taken mod 2^64; the combined columns equal the schoolbook
// columns, which the generator keeps below 2^64 (and the half sums below 2^32,
// check_xround), so the result is exact.
struct KAcc {
  uint64_t z0[9], z1[9], z2[9];
};
HG_DEV void kacc_mad_pinned(KAcc& k, const Fp& x, const Fp& y) {
  uint32_t sx[5], sy[5];
#pragma unroll
  for (int i = 0; i < 5; i++) {
    sx[i] = x.l[i] + x.l[i + 5];
    sy[i] = y.l[i] + y.l[i + 5];
  }
#pragma unroll
  for (int i = 0; i < 5; i++)
#pragma unroll
    for (int j = 0; j < 5; j++) {
      k.z0[i + j] += (uint64_t)x.l[i] * y.l[j];
      asm("" : "+v"(k.z0[i + j]));
      k.z2[i + j] += (uint64_t)x.l[i + 5] * y.l[j + 5];
      asm("" : "+v"(k.z2[i + j]));
      k.z1[i + j] += (uint64_t)sx[i] * sy[j];
      asm("" : "+v"(k.z1[i + j]));
    }
}
// FUSE: products 0 .. NP - 2 as above, the last one schoolbook with REDC
// digits 0..9 interleaved (acc_mad_redc), after the half products combined
template <int W, int NP, bool FUSE>
HG_DEV void x_products_ks(const Team& T, const uint32_t (&w)[W], int base, Acc& acc, Fp a, Fp b) {
  constexpr int NK = FUSE ? NP - 1 : NP;  // Karatsuba products
  KAcc k;
#pragma unroll
  for (int c = 0; c < 9; c++) k.z0[c] = k.z1[c] = k.z2[c] = 0;
  x_for<NK>([&](auto p) {
    Fp a2, b2;
    if constexpr (p + 1 < NP) {
      ld_fp_a8(a2, x_at(T, x_off(w, base + 2 * (p + 1))));
      ld_fp_a8(b2, x_at(T, x_off(w, base + 2 * (p + 1) + 1)));
    }
    kacc_mad_pinned(k, a, b);
#pragma unroll
    for (int c = 0; c < 9; c++) asm volatile("" : "+v"(k.z0[c]), "+v"(k.z1[c]), "+v"(k.z2[c]));
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (p + 1 < NP) {
      a = a2;
      b = b2;
    }
  });
#pragma unroll
  for (int c = 0; c < 9; c++) {
    acc.c[c] += k.z0[c];
    acc.c[c + 10] += k.z2[c];
    acc.c[c + 5] += k.z1[c] - (k.z0[c] + k.z2[c]);
  }
  if constexpr (FUSE) acc_mad_redc(acc, a, b);  // a, b: the last product's operands
}

// EF: a0, b0 already hold the first product's operands (read before the
// pre-pass: plain elements, see x_round)
template <int W, int NP, int NL, int KL, int KS, int LZ = 0, int EF = 0, int FU = 0>
HG_DEV void x_job(const Team& T, const uint32_t (&w)[W], int base, Fp& r, uint32_t& dst, Fp a0 = Fp{},
                  Fp b0 = Fp{}) {
  Acc acc;
  acc_zero(acc);
  constexpr int lbase = 2 * NP;
  // the linear terms' elements and the first product's operands are loaded
  // together, so the job pays one LDS round trip before its first mad
  Fp lx[NL > 0 ? NL : 1];
  if constexpr (NL > 0) x_for<NL>([&](auto t) { ld_fp_a8(lx[t], x_at(T, x_term_off(w, base + lbase + t))); });
  if constexpr (NP > 0 && !EF) {
    ld_fp_a8(a0, x_at(T, x_off(w, base)));
    ld_fp_a8(b0, x_at(T, x_off(w, base + 1)));
  }
  if constexpr (NL > 0) {
    uint32_t val[10];
    x_lincomb_sum<W, NL, KL>(w, base + lbase, lx, val);
#pragma unroll
    for (int l = 0; l < 10; l++) acc.c[kRedcSteps + l] = val[l];
  }
  constexpr bool FUSE = HG_REDC_FUSE && FU && NP > 0;
  constexpr int FROM = FUSE ? 10 : 0;  // REDC digits the products already ran
  if constexpr (KS) x_products_ks<W, NP, FUSE>(T, w, base, acc, a0, b0);
  else x_products<W, NP, FUSE>(T, w, base, acc, a0, b0);
  dst = x_off(w, base + lbase + NL);
  if constexpr (NL > 0 && LZ) acc_reduce_wide_lazy<FROM>(r, acc);  // linear terms, lazy: [0, 2p)
  else if constexpr (NL > 0) acc_reduce_wide<FROM>(r, acc);       // linear terms: result < 31p
  else acc_reduce<FROM>(r, acc);                                  // products only: < 2p, one subtraction
}

// A single-job round on a team spread over the kSplitWaves waves of a
// workgroup (Team::split): the products are cut into kSplitWaves contiguous
// ranges, wave r sums range r, the last wave also the linear terms; waves
// 1.. hand their 21 columns to wave 0 through LDS (T.xchg, the same lane of
// the other waves), wave 0 adds them and reduces. The column sums are those
// of x_job, so the result is the same value. Ends with the round's closing
// barrier.
template <int NP, int R>
struct XSplitRange {
  static constexpr int kQ = (NP + kSplitWaves - 1) / kSplitWaves;
  static constexpr int kLo = R * kQ < NP ? R * kQ : NP;
  static constexpr int kHi = (R + 1) * kQ < NP ? (R + 1) * kQ : NP;
  static constexpr int kN = kHi - kLo;
};
template <int W, int NP, int NL, int KL, int KS, int LZ, int EF>
HG_DEV void x_job_split(const Team& T, const uint32_t (&w)[W], int base, Fp a0, Fp b0) {
  constexpr int lbase = 2 * NP;
  constexpr int H = XSplitRange<NP, 0>::kN;  // wave 0's products
  // wave r > 0: its partial columns, if it has any work
  auto partial = [&](auto rr) {
    constexpr int R = decltype(rr)::value;
    using Rg = XSplitRange<NP, R>;
    constexpr bool kLin = R == kSplitWaves - 1 && NL > 0;
    if constexpr (Rg::kN > 0 || kLin) {
      Acc acc;
      acc_zero(acc);
      Fp lx[NL > 0 ? NL : 1];
      if constexpr (kLin) x_for<NL>([&](auto t) { ld_fp_a8(lx[t], x_at(T, x_term_off(w, base + lbase + t))); });
      Fp a, b;
      if constexpr (Rg::kN > 0) {
        ld_fp_a8(a, x_at(T, x_off(w, base + 2 * Rg::kLo)));
        ld_fp_a8(b, x_at(T, x_off(w, base + 2 * Rg::kLo + 1)));
      }
      if constexpr (NL > 0) {  // (NL first: the call below does not depend on R)
        if constexpr (kLin) {
          uint32_t val[10];
          x_lincomb_sum<W, NL, KL>(w, base + lbase, lx, val);
#pragma unroll
          for (int l = 0; l < 10; l++) acc.c[kRedcSteps + l] = val[l];
        }
      }
      if constexpr (KS && Rg::kN >= 3) x_products_ks<W, Rg::kN, false>(T, w, base + 2 * Rg::kLo, acc, a, b);
      else if constexpr (Rg::kN > 0) x_products<W, Rg::kN, false>(T, w, base + 2 * Rg::kLo, acc, a, b);
      uint4* x4 = (uint4*)__builtin_assume_aligned(T.xchg + (R - 1) * kXchgWords, 16);
#pragma unroll
      for (int c = 0; c < 10; c++)
        x4[c] = make_uint4((uint32_t)acc.c[2 * c], (uint32_t)(acc.c[2 * c] >> 32), (uint32_t)acc.c[2 * c + 1],
                           (uint32_t)(acc.c[2 * c + 1] >> 32));
      reinterpret_cast<uint64_t*>(T.xchg + (R - 1) * kXchgWords)[20] = acc.c[20];
    }
  };
  if (T.wave != 0) {
    if constexpr (kSplitWaves == 2) {
      partial(std::integral_constant<int, 1>{});
    } else {
      x_for<kSplitWaves - 1>([&](auto r) {
        constexpr int R = decltype(r)::value + 1;
        if (T.wave == R) partial(std::integral_constant<int, R>{});
      });
    }
    __syncthreads();  // A: the partial columns in LDS, every read of these waves done
    __syncthreads();  // the round's end
    return;
  }
  Acc acc;
  acc_zero(acc);
  if constexpr (H > 0) {
    if constexpr (!EF) {
      ld_fp_a8(a0, x_at(T, x_off(w, base)));
      ld_fp_a8(b0, x_at(T, x_off(w, base + 1)));
    }
    if constexpr (KS && H >= 3) x_products_ks<W, H, false>(T, w, base, acc, a0, b0);
    else x_products<W, H, false>(T, w, base, acc, a0, b0);
  }
  const uint32_t dst = x_off(w, base + lbase + NL);
  __syncthreads();  // A
  x_for<kSplitWaves - 1>([&](auto r) {
    constexpr int R = decltype(r)::value + 1;
    if constexpr (XSplitRange<NP, R>::kN > 0 || (R == kSplitWaves - 1 && NL > 0)) {
      const uint4* x4 = (const uint4*)__builtin_assume_aligned(T.xchg + (R - 1) * kXchgWords, 16);
#pragma unroll
      for (int c = 0; c < 10; c++) {
        const uint4 v = x4[c];
        acc.c[2 * c] += (uint64_t)v.x | ((uint64_t)v.y << 32);
        acc.c[2 * c + 1] += (uint64_t)v.z | ((uint64_t)v.w << 32);
      }
      acc.c[20] += reinterpret_cast<const uint64_t*>(T.xchg + (R - 1) * kXchgWords)[20];
    }
  });
  Fp r;
#ifdef HG_SPLIT_NOREDC  // timing probe only (wrong values): the reduction's share of the critical path
#pragma unroll
  for (int l = 0; l < 10; l++) r.l[l] = (uint32_t)acc.c[11 + l] & kMask;
#else
  if constexpr (NL > 0 && LZ) acc_reduce_wide_lazy<0>(r, acc);
  else if constexpr (NL > 0) acc_reduce_wide<0>(r, acc);
  else acc_reduce<0>(r, acc);
#endif
  if (dst != 0xffffu) st_fp_a8(x_at(T, dst), r.l);
  __syncthreads();  // the round's end
}

// Split teams' pre-pass: 1 = the waves share the values (a workgroup barrier
// before the products); 0 = every wave evaluates every value and stores it
// (the waves store identical words), so each wave reads back its own stores
// and a wave-level sync suffices. 0 measured slower: 0.768 vs 0.745 ms for 128
// checks (profiles/r05lv_split_prepass_ab.json) — the barrier is cheaper than
// the lincombs it saves on wave 0's path
#ifndef HG_SPLIT_PREPASS
#define HG_SPLIT_PREPASS 1
#endif
static constexpr bool kSplitPrepass = HG_SPLIT_PREPASS != 0;

// the pre-pass of a split team's round: wave r evaluates the values v = r,
// r + kSplitWaves, ...
template <int NV, int NT, int W, int KP>
HG_DEV void x_prepass_split(const Team& T, const uint32_t (&w)[W]) {
  auto part = [&](auto par) {
    constexpr int P = decltype(par)::value;
    constexpr int NH = (NV - P + kSplitWaves - 1) / kSplitWaves;  // values P, P + kSplitWaves, ...
    if constexpr (NH > 0) {
      Fp xs[NH][NT];
      x_for<NH>([&](auto h) {
        x_for<NT>([&](auto t) {
          ld_fp_a8(xs[h][t], x_at(T, x_term_off(w, (P + kSplitWaves * h) * (1 + NT) + 1 + t)));
        });
      });
      __builtin_amdgcn_sched_barrier(0);
      uint32_t val[NH][10];
      x_for<NH>([&](auto h) { x_lincomb_sum<W, NT, KP>(w, (P + kSplitWaves * h) * (1 + NT) + 1, xs[h], val[h]); });
      x_for<NH>([&](auto h) {
        const uint32_t dst = x_off(w, (P + kSplitWaves * h) * (1 + NT));
        if (dst != 0xffffu) st_fp_a8(x_at(T, dst), val[h]);
      });
    }
  };
  if constexpr (kSplitWaves == 2) {
    if (T.wave == 0) part(std::integral_constant<int, 0>{});
    else part(std::integral_constant<int, 1>{});
  } else {
    x_for<kSplitWaves>([&](auto r) {
      if (T.wave == decltype(r)::value) part(r);
    });
  }
}

// One round. Table layout per lane (16-bit entries): NV x (dst, NT x term),
// then job 1 (NP x (u, v), NL x term, dst) and, in a fused round (NP2 + NL2 >
// 0), job 2 (NP2 x (u, v), NL2 x term, dst2); padded to W dwords. Both jobs
// read before either result is stored, so in-place programs are fine.
// off: the round's table offset
template <int NV, int NT, int NP, int NL, int W, int NP2, int NL2, int KP, int KL1, int KL2, int KS1, int KS2, int LZ,
          int EF, int FU>
HG_DEV void x_round(const Team& T, XStream& S, int off, XHint nxt) {
  if (S.off != off) x_fetch(T, S, XHint{off, W});  // wave-uniform; only without a (correct) hint
  uint32_t w[W];
  x_for<W>([&](auto i) { w[i] = S.w[i]; });
  if (nxt.off >= 0) x_fetch(T, S, nxt);
  constexpr int jbase = NV * (1 + NT);
  // EF (generator): every lane's first product reads plain elements, so its
  // operands are read with the pre-pass's inputs and the products do not wait
  // for the pre-pass's stores to come back
  Fp e0, e1;
  if constexpr (EF) {
    ld_fp_a8(e0, x_at(T, x_off(w, jbase)));
    ld_fp_a8(e1, x_at(T, x_off(w, jbase + 1)));
  }
  if constexpr (NV > 0) {
    // every lane evaluates every combination (a lane without one reads the
    // ZERO register with coefficient 0: valid offsets, discarded result), and
    // the values are pinned before the first store, so the compiler cannot
    // sink a combination into its store's branch: the loads of all
    // combinations issue together instead of one LDS latency per combination
    if (kTeamSplit && kSplitPrepass && T.split) {  // a split team: the waves take turns over the values
      x_prepass_split<NV, NT, W, KP>(T, w);
      team_sync(T);
    } else {
    Fp xs[NV][NT];
    x_for<NV>([&](auto v) {
      x_for<NT>([&](auto t) { ld_fp_a8(xs[v][t], x_at(T, x_term_off(w, v * (1 + NT) + 1 + t))); });
    });
    __builtin_amdgcn_sched_barrier(0);  // every load of the pre-pass in flight before the first sum
    uint32_t val[NV][10];
    x_for<NV>([&](auto v) { x_lincomb_sum<W, NT, KP>(w, v * (1 + NT) + 1, xs[v], val[v]); });
#pragma unroll
    for (int v = 0; v < NV; v++)
#pragma unroll
      for (int l = 0; l < 10; l++) asm volatile("" : "+v"(val[v][l]));
    x_for<NV>([&](auto v) {
      const uint32_t dst = x_off(w, v * (1 + NT));
      if (dst != 0xffffu) st_fp_a8(x_at(T, dst), val[v]);
    });
    team_sync();
    }
  }
  if constexpr (kTeamSplit && NP2 == 0 && NL2 == 0) {
    if (T.split) {
      x_job_split<W, NP, NL, KL1, KS1, LZ, EF>(T, w, jbase, e0, e1);
      return;
    }
  }
  Fp r;
  uint32_t dst;
  if constexpr (EF) x_job<W, NP, NL, KL1, KS1, LZ, EF, FU>(T, w, jbase, r, dst, e0, e1);
  else x_job<W, NP, NL, KL1, KS1, LZ, 0, FU>(T, w, jbase, r, dst);
  if constexpr (NP2 > 0 || NL2 > 0) {
    Fp r2;
    uint32_t dst2;
    x_job<W, NP2, NL2, KL2, KS2>(T, w, jbase + 2 * NP + NL + 1, r2, dst2);
    team_sync(T);
    // a split team runs a fused round whole on both waves; wave 0 stores
    if (!kTeamSplit || !T.split || T.wave == 0) {
      if (dst != 0xffffu) st_fp_a8(x_at(T, dst), r.l);
      if (dst2 != 0xffffu) st_fp_a8(x_at(T, dst2), r2.l);
    }
  } else {
    team_sync(T);
    if (dst != 0xffffu) st_fp_a8(x_at(T, dst), r.l);
  }
  team_sync(T);
}

// ------------------------------------------------------------------ call-site wrappers
// Each takes the stream and a hint naming the program that runs next.
template <int D, int A, int B>
using IMul12 = XInst<XP_MUL12, D, A, B>;
template <int D, int A>
using ICyc = XInst<XP_CYC_SQR_X, D, A>;
template <int D, int A>
using ICyc0 = XInst<XP_CYC_SQR, D, A>;  // canonical result (CYC_SQR_X's is lazy)
template <int D, int A>
using ISqr12 = XInst<XP_SQR12, D, A>;
template <int D, int A>
using ILinePk = XInst<XP_LINE_PK, D, A>;
template <int D, int A>
using ILineFix = XInst<XP_LINE_FIX, D, A>;
template <int PROG>
using IG2 = XInst<PROG>;

// dst = a * b (Fp12)
template <int D, int A, int B>
HG_DEV void x_mul12(const Team& T, XStream& S, XHint h) { IMul12<D, A, B>::run(T, S, h); }
// dst = a^2 for a in the cyclotomic subgroup (Granger-Scott)
template <int D, int A>
HG_DEV void x_cyc_sqr(const Team& T, XStream& S, XHint h) { ICyc<D, A>::run(T, S, h); }
// dst = a^2 (Miller loop)
template <int D, int A>
HG_DEV void x_sqr12(const Team& T, XStream& S, XHint h) { ISqr12<D, A>::run(T, S, h); }
// dst = a * (LC + LB w + LA w^3) / a * (FC + FB w + FA w^3): the pk / G2Base lines
template <int D, int A>
HG_DEV void x_line_pk(const Team& T, XStream& S, XHint h) { ILinePk<D, A>::run(T, S, h); }
template <int D, int A>
HG_DEV void x_line_fix(const Team& T, XStream& S, XHint h) { ILineFix<D, A>::run(T, S, h); }
// G2 Miller-loop steps on the register file (x/crypto lineFunctionDouble / Add)
template <int PROG>
HG_DEV void x_g2(const Team& T, XStream& S, XHint h) { IG2<PROG>::run(T, S, h); }


// dst = a^v for a in the cyclotomic subgroup (a^-1 = conj(a)), where v =
// 1868033 = 2^21 - 2^18 + 2^15 + 2^8 + 1 is the cube root of the BN
// parameter u (u = v^3): 21 cyclotomic squarings and 4
// multiplications, scratch slot K = a^-1. h: the program that runs after it.
// The squaring runs are runtime loops (one copy of each program in the code:
// the final exponentiation is long enough to miss in the instruction cache).
template <int D, int SA>
HG_DEV void t12_pow_v_x(const Team& T, XStream& S, XHint h) {
  static_assert(D != SA && D != S_K && SA != S_K, "scratch slot");
  t12_conj(T, S_K, SA);                      // a^-1
  x_cyc_sqr<D, SA>(T, S, xh<ICyc<D, D>>());  // a^2
  // segments: squarings, then a multiplication by a^-1 (segment 0) or a:
  // a^2 -> a^8 -> a^7 -> a^56 -> a^57 -> a^7296 -> a^7297 -> a^(7297 * 256) -> a^v
  const int nsq[4] = {2, 3, 7, 8};
#pragma unroll 1
  for (int seg = 0; seg < 4; seg++) {
    const XHint mul = seg == 0 ? xh<IMul12<D, D, S_K>>() : xh<IMul12<D, D, SA>>();
#pragma unroll 1
    for (int i = 0; i < nsq[seg]; i++) x_cyc_sqr<D, D>(T, S, i + 1 < nsq[seg] ? xh<ICyc<D, D>>() : mul);
    if (seg == 0) x_mul12<D, D, S_K>(T, S, xh<ICyc<D, D>>());
    else x_mul12<D, D, SA>(T, S, seg < 3 ? xh<ICyc<D, D>>() : h);
  }
}

// dst = a^u (x/crypto gfP12.Exp(t, u)) for a in the cyclotomic subgroup:
// three exponentiations by v (u = v^3): 63 cyclotomic squarings and 12
// multiplications (a width-3 NAF of u needs 62 + 17). Scratch slots J, K
// (dst, SA not among them). h: the program that runs after it.
template <int D, int SA>
HG_DEV void t12_pow_u_x(const Team& T, XStream& S, XHint h) {
  static_assert(D != S_J && D != S_K && SA != S_J && SA != S_K && D != SA, "scratch slots");
  t12_pow_v_x<D, SA>(T, S, xh<ICyc<S_J, D>>());
  t12_pow_v_x<S_J, D>(T, S, xh<ICyc<D, S_J>>());
  t12_pow_v_x<D, S_J>(T, S, h);
}

// dst = a^-1 (x/crypto gfP12.Invert) with scratch slots S1, S2
template <int DST, int SA, int S1, int S2>
HG_DEV void t12_inv_x(const Team& T, XStream& S, XHint h) {
  t12_conj(T, S1, SA);                                       // S1 = conj(a)
  x_mul12<S2, SA, S1>(T, S, xh<IMul12<DST, S1, S2>>());      // S2 = a conj(a) = N (even coefficients only)
  t12_inv_norm(T, S2);                                       // S2 = N^-1
  x_mul12<DST, S1, S2>(T, S, h);                             // conj(a) / N
}

// ------------------------------------------------------------------ layout S (k_verify_sig)
// The same programs bound to k_verify_sig's compact team region: slots F..G
// only, registers at kSigRegBase (tools/gen_g2_schedule.py SIG_INSTANCES).
template <int D, int A, int B>
using IMul12S = XInst<XP_MUL12_S, D, A, B>;
template <int D, int A>
using ICycS = XInst<XP_CYC_SQR_X_S, D, A>;

}  // namespace hg
