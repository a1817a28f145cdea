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

__device__ uint64_t g_ticks[1024];

// fill the team's LDS with reduced random-looking elements
HG_DEV void fill(uint32_t* lds, int words, uint32_t seed) {
  for (int i = threadIdx.x; i < words; i += 64) {
    uint32_t v = (uint32_t)(i * 2654435761u) ^ seed;
    lds[i] = ((i % 10) == 9) ? (v & 0x3fffffu) : (v & kMask);
  }
  __syncthreads();
}

template <int OP>
__global__ __launch_bounds__(64) void k_op(uint32_t seed, uint32_t* sink) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[kTeamsPerBlock * kTeamWords];
  fill(lds, kTeamsPerBlock * kTeamWords, seed + blockIdx.x);
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
    if constexpr (OP == 7) g2_program(T, F, kProgDBL);
    if constexpr (OP == 8) g2_program(T, F, kProgADD_POS);
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
  if (threadIdx.x == 0) g_ticks[blockIdx.x] = t1 - t0;
  if (lds[threadIdx.x] == 0x12345678u) sink[0] = 1;
}

static const char* kNames[] = {"t12_mul", "t12_sqr_fast", "t12_cyc_sqr", "t12_mul_line", "t12_frob", "t12_frob2",
                               "t12_conj", "g2_double", "g2_add", "fp_inv", "x_cyc_sqr", "x_mul12", "x_sqr12",
                               "x_line_pk", "x_g2_dbl", "x_g2_add"};

template <int OP>
void run(uint32_t* sink) {
  k_op<OP><<<1024, 64>>>(7, sink);
  (void)hipDeviceSynchronize();
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  k_op<OP><<<1024, 64>>>(11, sink);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  std::vector<uint64_t> t(1024);
  (void)hipMemcpyFromSymbol(t.data(), HIP_SYMBOL(g_ticks), 1024 * 8, 0, hipMemcpyDeviceToHost);
  double s = 0;
  for (auto v : t) s += (double)v;
  printf("{\"op\": \"%s\", \"ticks_per_op\": %.0f, \"kernel_us\": %.1f}\n", kNames[OP], s / 1024 / REPS, ms * 1e3);
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
  run<7>(sink);
  run<8>(sink);
  run<9>(sink);
  run<10>(sink);
  run<11>(sink);
  run<12>(sink);
  run<13>(sink);
  run<14>(sink);
  run<15>(sink);
  (void)hipFree(sink);
  return 0;
}
