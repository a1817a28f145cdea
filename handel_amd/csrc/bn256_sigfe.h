// bn256_sigfe.h — the sig-only pairing kernels' final exponentiation on their
// compact team regions: k_verify_sig (16-lane teams, layout S, bn256_gt.hip)
// and k_verify_sig12 (12-lane teams, layout T, bn256_sig12.hip) run the same
// Fuentes-Castaneda chain, each on its own bound program tables
// (tools/gen_g2_schedule.py SIG_INSTANCES, SIG_T_INSTANCES).
// P names the two programs: P::Mul<D, A, B> (D = A * B) and P::Cyc<D, A>
// (D = A^2 in the cyclotomic subgroup, lazy result).
#pragma once
#include "bn256_xprog.h"

namespace hg {

// 16-lane teams: the programs' pre-pass values on lanes 0..15
struct SigProgs16 {
  template <int D, int A, int B>
  using Mul = XInst<XP_MUL12_S, D, A, B>;
  template <int D, int A>
  using Cyc = XInst<XP_CYC_SQR_X_S, D, A>;
};
// 12-lane teams (five per wave, layout T): every pre-pass value on lanes 0..11
struct SigProgs12 {
  template <int D, int A, int B>
  using Mul = XInst<XP_MUL12_12_T, D, A, B>;
  template <int D, int A>
  using Cyc = XInst<XP_CYC_SQR_X_12_T, D, A>;
};

// An Fp12 value parked in HBM while the team region is short of slots: lane
// e < 12 moves its own element (40 bytes) of slot s to / from `park` (a Gt
// record of this check; the written lines are never read by another lane, and
// the caller's fence orders the stores before the later loads).
HG_DEV void t12_park(const Team& T, int s, uint32_t* park) {
  Fp v;
  ld_fp_a8(v, slot(T, s) + T.e * 10);
  if (T.active) {
    uint2* dst = (uint2*)__builtin_assume_aligned(park + 10 * T.e, 8);
#pragma unroll
    for (int i = 0; i < 5; i++) dst[i] = make_uint2(v.l[2 * i], v.l[2 * i + 1]);
  }
  __threadfence_block();
}
HG_DEV void t12_unpark(const Team& T, int s, const uint32_t* park) {
  const uint2* src = (const uint2*)__builtin_assume_aligned(park + 10 * T.e, 8);
  uint32_t v[10];
#pragma unroll
  for (int i = 0; i < 5; i++) {
    const uint2 x = src[i];
    v[2 * i] = x.x;
    v[2 * i + 1] = x.y;
  }
  if (T.active) st_fp_a8(slot(T, s) + T.e * 10, v);
  team_sync(T);
}

template <class P>
struct SigFE {
  template <int D, int A, int B>
  using IMul12S = typename P::template Mul<D, A, B>;
  template <int D, int A>
  using ICycS = typename P::template Cyc<D, A>;

  // t12_pow_v_x (bn256_xprog.h) on layout S: dst = a^v with the conjugate of
  // a in slot SK (v = 1868033, u = v^3)
  template <int D, int SA, int SK>
  HG_DEV static void t12_pow_v_s(const Team& T, XStream& S, XHint h) {
    static_assert(D != SA && D != SK && SA != SK, "scratch slot");
    t12_conj(T, SK, SA);                            // a^-1
    ICycS<D, SA>::run(T, S, xh<ICycS<D, D>>());    // a^2
    const int nsq[4] = {2, 3, 7, 8};
#pragma unroll 1
    for (int seg = 0; seg < 4; seg++) {
      const XHint mul = seg == 0 ? xh<IMul12S<D, D, SK>>() : xh<IMul12S<D, D, SA>>();
#pragma unroll 1
      for (int i = 0; i < nsq[seg]; i++) ICycS<D, D>::run(T, S, i + 1 < nsq[seg] ? xh<ICycS<D, D>>() : mul);
      if (seg == 0) IMul12S<D, D, SK>::run(T, S, xh<ICycS<D, D>>());
      else IMul12S<D, D, SA>::run(T, S, seg < 3 ? xh<ICycS<D, D>>() : h);
    }
  }

  // team_final_exp_fc (bn256_pairing.h) on layout S: the same chain over seven
  // slots F, A, B, C, D, E, G (the full layout spreads it over eleven), so the
  // team region is 118 elements instead of 180. Slot roles: F = res; the easy
  // part's inversion uses D, E; the exponentiations by v ping-pong D <-> E
  // with the base's conjugate in G; t0 = A, t1 = B, t2 = C, t4 = G, t3 = B
  // (once t1 is consumed); D carries the Frobenius temporaries of the last
  // products. The next base t2^2 is a product, not the canonical cyclotomic
  // squaring, whose pre-pass scratch would end the region 2 elements later.
  HG_DEV static constexpr XHint final_exp_hint_s() { return xh<IMul12S<S_E, S_F, S_D>>(); }
  HG_DEV static void team_final_exp_fc_s(const Team& T, XStream& S) {
    // easy part: res = f^((p^6 - 1)(p^2 + 1)), f^-1 = conj(f) / (f conj(f))
    t12_conj(T, S_D, S_F);
    IMul12S<S_E, S_F, S_D>::run(T, S, xh<IMul12S<S_A, S_D, S_E>>());  // N = f conj(f)
    t12_inv_norm(T, S_E);                                              // N^-1
    IMul12S<S_A, S_D, S_E>::run(T, S, xh<IMul12S<S_F, S_B, S_A>>());  // A = f^-1
    t12_conj(T, S_B, S_F);
    IMul12S<S_F, S_B, S_A>::run(T, S, xh<IMul12S<S_F, S_F, S_A>>());  // f^(p^6 - 1)
    t12_frob2(T, S_A, S_F);
    IMul12S<S_F, S_F, S_A>::run(T, S, xh<ICycS<S_E, S_D>>());         // res
    t12_copy(T, S_D, S_F);  // base of the first exponentiation
#pragma unroll 1
    for (int ph = 0; ph < 3; ph++) {
#pragma unroll 1
      for (int st = 0; st < 3; st++) {  // E = D^v, D = E^v, E = D^v
        const XHint next = st < 2 ? ((st & 1) ? xh<ICycS<S_E, S_D>>() : xh<ICycS<S_D, S_E>>())
                                  : (ph == 0 ? xh<ICycS<S_A, S_A>>() : ph == 1 ? xh<IMul12S<S_B, S_C, S_G>>()
                                                                               : xh<IMul12S<S_G, S_B, S_E>>());
        if ((st & 1) == 0) t12_pow_v_s<S_E, S_D, S_G>(T, S, next);
        else t12_pow_v_s<S_D, S_E, S_G>(T, S, next);
      }
      if (ph == 0) {  // t0 = conj(res^u)^2, t1 = t0^2 t0; next base t1
        t12_conj(T, S_A, S_E);
        ICycS<S_A, S_A>::run(T, S, xh<ICycS<S_B, S_A>>());
        ICycS<S_B, S_A>::run(T, S, xh<IMul12S<S_B, S_A, S_B>>());
        IMul12S<S_B, S_A, S_B>::run(T, S, xh<ICycS<S_E, S_D>>());
        t12_copy(T, S_D, S_B);
      } else if (ph == 1) {  // t2 = conj(t1^u), t1 = t2 conj(t1); next base t3 = t2^2
        t12_conj(T, S_C, S_E);
        t12_conj(T, S_G, S_B);
        IMul12S<S_B, S_C, S_G>::run(T, S, xh<IMul12S<S_D, S_C, S_C>>());
        IMul12S<S_D, S_C, S_C>::run(T, S, xh<ICycS<S_E, S_D>>());  // canonical (feeds a conj)
      } else {  // t4 = t1 t3^u
        IMul12S<S_G, S_B, S_E>::run(T, S, xh<IMul12S<S_B, S_A, S_G>>());
      }
    }
    IMul12S<S_B, S_A, S_G>::run(T, S, xh<IMul12S<S_A, S_C, S_G>>());  // t3 = t0 t4
    IMul12S<S_A, S_C, S_G>::run(T, S, xh<IMul12S<S_A, S_F, S_A>>());  // t0 = t2 t4
    IMul12S<S_A, S_F, S_A>::run(T, S, xh<IMul12S<S_A, S_D, S_A>>());  // t0 = res t0
    t12_frob(T, S_D, S_B);
    IMul12S<S_A, S_D, S_A>::run(T, S, xh<IMul12S<S_A, S_D, S_A>>());  // t0 = frob(t3) t0
    t12_frob2(T, S_D, S_G);
    IMul12S<S_A, S_D, S_A>::run(T, S, xh<IMul12S<S_D, S_D, S_B>>());  // t0 = frob2(t4) t0
    t12_conj(T, S_D, S_F);
    IMul12S<S_D, S_D, S_B>::run(T, S, xh<IMul12S<S_F, S_D, S_A>>());  // t2 = conj(res) t3
    t12_frob(T, S_D, S_D);
    t12_frob2(T, S_D, S_D);                                            // t2 = frob^3(t2)
    IMul12S<S_F, S_D, S_A>::run(T, S, xh_none());                      // result
  }

  // The same chain on FIVE slots F, A, B, C, D (layout T, k_verify_sig12):
  // res (park0) and t0 (park1) wait in HBM while the exponentiations by u
  // run, so no more than five values are ever live in the team region. The
  // exponentiations by v ping-pong C <-> D with the base's conjugate in B
  // (phase 0) or F (phases 1, 2); t1 = B, t2 = A, t4 = D; the final products
  // accumulate in F. The result lands in F.
  HG_DEV static constexpr XHint final_exp_hint_t() { return xh<IMul12S<S_B, S_F, S_D>>(); }
  // park(k): this check's parking record k (0: res, 1: t0), a callable so the
  // kernel can recompute the addresses instead of holding them in registers
  template <class Park>
  HG_DEV static void team_final_exp_fc_t(const Team& T, XStream& S, Park park) {
    fe_t_norm(T, S, fe_t_rest_hint());
    t12_inv_norm(T, S_B);  // N^-1
    fe_t_rest(T, S, park);
  }
  // the chain's first part, up to the norm: D = conj(f), B = N = f conj(f)
  // (the split kernels of bn256_sig12.hip end here and invert the norms of a
  // whole batch at once)
  HG_DEV static void fe_t_norm(const Team& T, XStream& S, XHint h) {
    // easy part: res = f^((p^6 - 1)(p^2 + 1)), f^-1 = conj(f) / (f conj(f))
    t12_conj(T, S_D, S_F);
    IMul12S<S_B, S_F, S_D>::run(T, S, h);  // N = f conj(f)
  }
  HG_DEV static constexpr XHint fe_t_rest_hint() { return xh<IMul12S<S_A, S_D, S_B>>(); }
  // the rest, with f in F, conj(f) in D and N^-1 in B
  template <class Park>
  HG_DEV static void fe_t_rest(const Team& T, XStream& S, Park park) {
    IMul12S<S_A, S_D, S_B>::run(T, S, xh<IMul12S<S_F, S_B, S_A>>());  // A = f^-1
    t12_conj(T, S_B, S_F);
    IMul12S<S_F, S_B, S_A>::run(T, S, xh<IMul12S<S_F, S_F, S_A>>());  // f^(p^6 - 1)
    t12_frob2(T, S_A, S_F);
    IMul12S<S_F, S_F, S_A>::run(T, S, xh<ICycS<S_C, S_F>>());         // res
    t12_park(T, S_F, park(0));
    // phase 0: C = res^u (res stays in F through the first exponentiation by v)
    t12_pow_v_s<S_C, S_F, S_B>(T, S, xh<ICycS<S_D, S_C>>());
    t12_pow_v_s<S_D, S_C, S_B>(T, S, xh<ICycS<S_C, S_D>>());
    t12_pow_v_s<S_C, S_D, S_B>(T, S, xh<ICycS<S_A, S_A>>());
    // t0 = conj(res^u)^2, t1 = t0^2 t0
    t12_conj(T, S_A, S_C);
    ICycS<S_A, S_A>::run(T, S, xh<ICycS<S_B, S_A>>());
    ICycS<S_B, S_A>::run(T, S, xh<IMul12S<S_B, S_A, S_B>>());
    IMul12S<S_B, S_A, S_B>::run(T, S, xh<ICycS<S_C, S_B>>());
    t12_park(T, S_A, park(1));
    // phase 1: C = t1^u (t1 stays in B)
    t12_pow_v_s<S_C, S_B, S_F>(T, S, xh<ICycS<S_D, S_C>>());
    t12_pow_v_s<S_D, S_C, S_F>(T, S, xh<ICycS<S_C, S_D>>());
    t12_pow_v_s<S_C, S_D, S_F>(T, S, xh<IMul12S<S_B, S_A, S_F>>());
    // t2 = conj(t1^u), t1 = t2 conj(t1); next base t3 = t2^2
    t12_conj(T, S_A, S_C);
    t12_conj(T, S_F, S_B);
    IMul12S<S_B, S_A, S_F>::run(T, S, xh<IMul12S<S_D, S_A, S_A>>());
    IMul12S<S_D, S_A, S_A>::run(T, S, xh<ICycS<S_C, S_D>>());  // canonical (feeds a conj)
    // phase 2: C = t3^u
    t12_pow_v_s<S_C, S_D, S_F>(T, S, xh<ICycS<S_D, S_C>>());
    t12_pow_v_s<S_D, S_C, S_F>(T, S, xh<ICycS<S_C, S_D>>());
    t12_pow_v_s<S_C, S_D, S_F>(T, S, xh<IMul12S<S_D, S_B, S_C>>());
    IMul12S<S_D, S_B, S_C>::run(T, S, xh<IMul12S<S_B, S_F, S_D>>());  // t4 = t1 t3^u
    t12_unpark(T, S_F, park(1));                                         // t0
    IMul12S<S_B, S_F, S_D>::run(T, S, xh<IMul12S<S_F, S_A, S_D>>());  // t3 = t0 t4
    IMul12S<S_F, S_A, S_D>::run(T, S, xh<IMul12S<S_F, S_A, S_F>>());  // t0 = t2 t4
    t12_unpark(T, S_A, park(0));                                         // res
    IMul12S<S_F, S_A, S_F>::run(T, S, xh<IMul12S<S_F, S_C, S_F>>());  // t0 = res t0
    t12_frob(T, S_C, S_B);
    IMul12S<S_F, S_C, S_F>::run(T, S, xh<IMul12S<S_F, S_C, S_F>>());  // t0 = frob(t3) t0
    t12_frob2(T, S_C, S_D);
    IMul12S<S_F, S_C, S_F>::run(T, S, xh<IMul12S<S_C, S_C, S_B>>());  // t0 = frob2(t4) t0
    t12_conj(T, S_C, S_A);
    IMul12S<S_C, S_C, S_B>::run(T, S, xh<IMul12S<S_F, S_C, S_F>>());  // t2 = conj(res) t3
    t12_frob(T, S_C, S_C);
    t12_frob2(T, S_C, S_C);                                            // t2 = frob^3(t2)
    IMul12S<S_F, S_C, S_F>::run(T, S, xh_none());                      // result
  }
};

}  // namespace hg
