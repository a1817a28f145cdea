// Per-building-block cost of the team ops of k_verify, measured in isolation
// under k_verify's launch shape (1024 single-wave workgroups of 4 teams = one
// wave per SIMD, the same LDS footprint). Each kernel runs one op REPS times;
// lane 0 of every block records s_memtime (shader-clock ticks) around the
// loop. Prints one JSON line per op: mean ticks per op per wave.
//
// Diagnostic tool (not part of the product). Build:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Ihandel_amd/csrc tools/opcycles.hip -o tools/opcycles
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "bn256_pairing.h"
#include "bn256_xprog.h"

using namespace hg;

#define REPS 16

static constexpr int kMaxBlocks = 2048;
__device__ uint64_t g_ticks[kMaxBlocks];

// fill the team's LDS with reduced random-looking elements
HG_DEV void fill(uint32_t* lds, int words, uint32_t seed) {
  for (int i = threadIdx.x; i < words; i += blockDim.x) {
    uint32_t v = (uint32_t)(i * 2654435761u) ^ seed;
    lds[i] = ((i % 10) == 9) ? (v & 0x3fffffu) : (v & kMask);
  }
  __syncthreads();
}

template <int OP, int TEAMS>
__global__ __launch_bounds__(64) void k_op(uint32_t seed, uint32_t* sink) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[TEAMS * kTeamWords];
  fill(lds, TEAMS * kTeamWords, seed + blockIdx.x);
  Team T = make_team(lds, kTeamWords);
  uint32_t* F = team_regs(T);
  if (T.tl == 0) {
    Fp z, o;
    fp_zero(z);
    fp_one(o);
    st_fp(F + R_ZERO * 10, z);
    st_fp(F + R_ONE * 10, o);
  }
  __syncthreads();
  XStream S = x_stream();  // each repetition prefetches the next one's table words
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < REPS; r++) {
    if constexpr (OP == 0) t12_mul(T, S_A, S_A, S_B);
    if constexpr (OP == 1) t12_sqr_fast(T, S_A, S_A);
    if constexpr (OP == 2) t12_cyc_sqr(T, S_A, S_A);
    if constexpr (OP == 3) t12_mul_line_regs(T, S_A, S_A, F, R_LA_x, R_LA_x + 2, R_LA_x + 4);
    if constexpr (OP == 4) t12_frob(T, S_A, S_A);
    if constexpr (OP == 5) t12_frob2(T, S_A, S_A);
    if constexpr (OP == 6) t12_conj(T, S_A, S_A);
    // OP 7, 8 (the Jacobian cross-check programs) use registers past the
    // kernels' register file: not measured
    if constexpr (OP == 10) x_cyc_sqr<S_A, S_A>(T, S, xh<ICyc<S_A, S_A>>());
    if constexpr (OP == 11) x_mul12<S_A, S_A, S_B>(T, S, xh<IMul12<S_A, S_A, S_B>>());
    if constexpr (OP == 12) x_sqr12<S_A, S_A>(T, S, xh<ISqr12<S_A, S_A>>());
    if constexpr (OP == 13) x_line_pk<S_A, S_A>(T, S, xh<ILinePk<S_A, S_A>>());
    if constexpr (OP == 14) x_g2<XP_PDBL>(T, S, xh<IG2<XP_PDBL>>());
    if constexpr (OP == 15) x_g2<XP_PADD_POS>(T, S, xh<IG2<XP_PADD_POS>>());
    if constexpr (OP == 9) {
      Fp v;
      ld_fp(v, slot(T, S_A) + T.e * 10);
      fp_inv(v, v);
      if (T.active) st_fp(slot(T, S_A) + T.e * 10, v);
    }
  }
  __syncthreads();
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0 && blockIdx.x < kMaxBlocks) g_ticks[blockIdx.x] = t1 - t0;
  if (lds[threadIdx.x] == 0x12345678u) sink[0] = 1;
}


// ---------------------------------------------------------------- 2-wave split prototype
// One round of a non-fused team program with its products split across the
// two waves of a 128-thread workgroup (wave w holds the same 4 teams' lanes):
// pre-pass value v by wave v % 2; products [0, NA) on wave 0, [NA, NP) on
// wave 1, whose 64-bit partial columns go through LDS (xch) to wave 0, which
// adds them, reduces and stores. Measures whether a second co-resident wave
// that takes half the products pays for the exchange.
template <int W, int P0, int P1>
HG_DEV void x_products_range(const Team& T, const uint32_t (&w)[W], int base, Acc& acc) {
  if constexpr (P1 > P0) {
    Fp a, b;
    ld_fp_a8(a, x_at(T, x_off(w, base + 2 * P0)));
    ld_fp_a8(b, x_at(T, x_off(w, base + 2 * P0 + 1)));
    x_for<P1 - P0>([&](auto q) {
      constexpr int p = P0 + q;
      Fp a2, b2;
      if constexpr (p + 1 < P1) {
        ld_fp_a8(a2, x_at(T, x_off(w, base + 2 * (p + 1))));
        ld_fp_a8(b2, x_at(T, x_off(w, base + 2 * (p + 1) + 1)));
      }
      acc_mad_pinned(acc, a, b);
#pragma unroll
      for (int c = 0; c < 21; c++) asm volatile("" : "+v"(acc.c[c]));
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (p + 1 < P1) {
        a = a2;
        b = b2;
      }
    });
  }
}

template <int NV, int NT, int NP, int NL, int W, int OFF, int KP, int KL1>
HG_DEV void x_round_split(const Team& T, XStream& S, XHint nxt, int wave, uint64_t* xch) {
  if (S.off != OFF) x_fetch(T, S, XHint{OFF, W});
  uint32_t w[W];
  x_for<W>([&](auto i) { w[i] = S.w[i]; });
  if (nxt.off >= 0) x_fetch(T, S, nxt);
  if constexpr (NV > 0) {
    x_for<NV>([&](auto v) {
      if ((v & 1) == wave) {
        constexpr int base = v * (1 + NT);
        const uint32_t dst = x_off(w, base);
        uint32_t val[10];
        x_lincomb<W, NT, KP>(T, w, base + 1, val);
        if (dst != 0xffffu) st_fp_a8(x_at(T, dst), val);
      }
    });
    __syncthreads();
  }
  constexpr int jbase = NV * (1 + NT);
  constexpr int NA = (NP + 1) / 2;
  Acc acc;
  acc_zero(acc);
  uint64_t* mine = xch + T.tl * 22;  // this team's exchange area, 22 u64 per lane
  if (wave == 0) {
    if constexpr (NL > 0) {
      uint32_t val[10];
      x_lincomb<W, NL, KL1>(T, w, jbase + 2 * NP, val);
#pragma unroll
      for (int l = 0; l < 10; l++) acc.c[kRedcSteps + l] = val[l];
    }
    x_products_range<W, 0, NA>(T, w, jbase, acc);
  } else {
    x_products_range<W, NA, NP>(T, w, jbase, acc);
#pragma unroll
    for (int c = 0; c < 21; c++) mine[c] = acc.c[c];
  }
  __syncthreads();
  if (wave == 0) {
#pragma unroll
    for (int c = 0; c < 21; c++) acc.c[c] += mine[c];
    Fp r;
    if constexpr (NL > 0) acc_reduce_wide(r, acc);
    else acc_reduce(r, acc);
    const uint32_t dst = x_off(w, jbase + 2 * NP + NL);
    if (dst != 0xffffu) st_fp_a8(x_at(T, dst), r.l);
  }
  __syncthreads();
}

// OP 16: x_mul12 (A = A * B), OP 17: x_cyc_sqr (A = A^2), split over two waves
template <int OP>
__global__ __launch_bounds__(128) void k_op2(uint32_t seed, uint32_t* sink) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[4 * kTeamWords];
  fill(lds, 4 * kTeamWords, seed + blockIdx.x);
  const int wave = threadIdx.x >> 6;
  Team T;
  {
    const int team = (threadIdx.x & 63) >> 4;
    T.tl = threadIdx.x & 15;
    T.base = lds + team * kTeamWords;
    T.active = T.tl < 12;
    T.e = T.active ? T.tl : 11;
    T.k = T.e >> 1;
    T.comp = T.e & 1;
  }
  uint32_t* F = team_regs(T);
  if (T.tl == 0 && wave == 0) {
    Fp z, o;
    fp_zero(z);
    fp_one(o);
    st_fp(F + R_ZERO * 10, z);
    st_fp(F + R_ONE * 10, o);
  }
  __syncthreads();
  // exchange area: slots G..L of each team's region (unused by these ops)
  uint64_t* xch = (uint64_t*)__builtin_assume_aligned(T.base + S_G * kFp12Words, 8);
  XStream S = x_stream();
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < REPS; r++) {
    if constexpr (OP == 16)
      x_round_split<2, 2, 12, 0, 16, IMul12<S_A, S_A, S_B>::kOff, 4, 0>(T, S, xh<IMul12<S_A, S_A, S_B>>(), wave, xch);
    if constexpr (OP == 17)
      x_round_split<2, 2, 3, 1, 7, ICyc<S_A, S_A>::kOff, 0, 6>(T, S, xh<ICyc<S_A, S_A>>(), wave, xch);
  }
  __syncthreads();
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0 && blockIdx.x < kMaxBlocks) g_ticks[blockIdx.x] = t1 - t0;
  if (lds[threadIdx.x] == 0x12345678u) sink[0] = 1;
}

static const char* kNames[] = {"t12_mul", "t12_sqr_fast", "t12_cyc_sqr", "t12_mul_line", "t12_frob", "t12_frob2",
                               "t12_conj", "g2_double", "g2_add", "fp_inv", "x_cyc_sqr", "x_mul12", "x_sqr12",
                               "x_line_pk", "x_g2_dbl", "x_g2_add", "x_mul12_split2", "x_cyc_sqr_split2"};

// TEAMS = 4: 1024 single-wave blocks of 4 teams = one wave per SIMD
// (k_verify's shape). TEAMS = 2: 2048 blocks of 2 teams (32 lanes, half the
// LDS) = two waves per SIMD, twice the wave-instructions for the same 4096
// teams: kernel_us(2) / kernel_us(4) = 2 / (issue-rate gain of a second
// co-resident wave) on this op's real instruction stream.
template <int OP, int TEAMS>
void run1(uint32_t* sink) {
  const int blocks = 4096 / TEAMS;
  k_op<OP, TEAMS><<<blocks, 16 * TEAMS>>>(7, sink);
  (void)hipDeviceSynchronize();
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  k_op<OP, TEAMS><<<blocks, 16 * TEAMS>>>(11, sink);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  std::vector<uint64_t> t(kMaxBlocks);
  (void)hipMemcpyFromSymbol(t.data(), HIP_SYMBOL(g_ticks), kMaxBlocks * 8, 0, hipMemcpyDeviceToHost);
  double s = 0;
  for (int b = 0; b < blocks; b++) s += (double)t[b];
  printf("{\"op\": \"%s\", \"teams_per_wave\": %d, \"ticks_per_op\": %.0f, \"kernel_us\": %.1f}\n", kNames[OP],
         TEAMS, s / blocks / REPS, ms * 1e3);
}
template <int OP>
void run(uint32_t* sink) {
  run1<OP, 4>(sink);
  run1<OP, 2>(sink);
}

template <int OP>
void run_split(uint32_t* sink) {
  const int blocks = 1024;  // 4 teams per workgroup of 2 waves: two waves per SIMD
  k_op2<OP><<<blocks, 128>>>(7, sink);
  (void)hipDeviceSynchronize();
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  k_op2<OP><<<blocks, 128>>>(11, sink);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  std::vector<uint64_t> t(kMaxBlocks);
  (void)hipMemcpyFromSymbol(t.data(), HIP_SYMBOL(g_ticks), kMaxBlocks * 8, 0, hipMemcpyDeviceToHost);
  double s = 0;
  for (int b = 0; b < blocks; b++) s += (double)t[b];
  printf("{\"op\": \"%s\", \"teams_per_wave\": 4, \"waves_per_team\": 2, \"ticks_per_op\": %.0f, \"kernel_us\": %.1f}\n",
         kNames[OP], s / blocks / REPS, ms * 1e3);
}

int main() {
  uint32_t* sink;
  (void)hipMalloc(&sink, 64);
  run<0>(sink);
  run<1>(sink);
  run<2>(sink);
  run<3>(sink);
  run<4>(sink);
  run<5>(sink);
  run<6>(sink);
  run<9>(sink);
  run<10>(sink);
  run<11>(sink);
  run<12>(sink);
  run<13>(sink);
  run<14>(sink);
  run<15>(sink);
  run_split<16>(sink);
  run_split<17>(sink);
  (void)hipFree(sink);
  return 0;
}
