// Integer / fp64 VALU throughput microbenchmark for gfx950.
// Measures the peak issue rate of the instructions a 256-bit Montgomery
// multiplier is built from, so the roofline in bench.py uses a measured
// P_mad instead of a datasheet guess.
//
// Build: hipcc --offload-arch=gfx950 -O3 tools/intrate.hip -o tools/intrate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define ITERS 4096
#define NACC 8

template <int OP>
__global__ __launch_bounds__(256) void k_rate(uint32_t* out, uint32_t seed) {
  uint32_t a = seed ^ threadIdx.x, b = seed * 2654435761u + blockIdx.x;
  uint64_t acc[NACC];
  uint32_t acc32[NACC];
  double accd[NACC];
#pragma unroll
  for (int i = 0; i < NACC; i++) {
    acc[i] = a + i;
    acc32[i] = b + i;
    accd[i] = (double)(a + i);
  }
  double da = (double)a * 1e-9, db = (double)b * 1e-9;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < NACC; i++) {
      if (OP == 0) {  // v_mad_u64_u32
        acc[i] = (uint64_t)(uint32_t)acc[i] * (uint64_t)(a + i) + (acc[i] >> 32);
      } else if (OP == 1) {  // v_mul_lo_u32
        acc32[i] = acc32[i] * (a + i) + 0;
      } else if (OP == 2) {  // v_mul_hi_u32
        acc32[i] = __umulhi(acc32[i], a + i);
      } else if (OP == 3) {  // v_mad_u32_u24
        acc32[i] = __umul24(acc32[i], a) + acc32[i];
      } else if (OP == 4) {  // v_add_co_u32 / v_addc chain (64-bit add)
        acc[i] = acc[i] + (uint64_t)(a + i) * 0x100000001ull;
      } else if (OP == 5) {  // v_fma_f64
        accd[i] = __fma_rn(accd[i], da, db);
      } else if (OP == 6) {  // v_add_u32
        acc32[i] = acc32[i] + (a ^ i);
      }
    }
  }
  uint64_t s = 0;
#pragma unroll
  for (int i = 0; i < NACC; i++) s += acc[i] + acc32[i] + (uint64_t)accd[i];
  if (s == 0x12345) out[0] = (uint32_t)s;
}

template <int OP>
double run(int blocks, uint32_t* d) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  k_rate<OP><<<blocks, 256>>>(d, 7);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  const int R = 5;
  for (int r = 0; r < R; r++) k_rate<OP><<<blocks, 256>>>(d, 7 + r);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  double ops = (double)R * blocks * 256.0 * ITERS * NACC;
  return ops / (ms * 1e-3) / 1e12;  // T ops/s
}

int main() {
  uint32_t* d;
  hipMalloc(&d, 64);
  const char* names[] = {"v_mad_u64_u32", "v_mul_lo_u32", "v_mul_hi_u32", "v_mad_u32_u24",
                         "add64(add_co+addc)", "v_fma_f64", "v_add_u32"};
  for (int blocks : {1024, 4096, 16384}) {
    double r[7];
    r[0] = run<0>(blocks, d);
    r[1] = run<1>(blocks, d);
    r[2] = run<2>(blocks, d);
    r[3] = run<3>(blocks, d);
    r[4] = run<4>(blocks, d);
    r[5] = run<5>(blocks, d);
    r[6] = run<6>(blocks, d);
    for (int i = 0; i < 7; i++)
      printf("{\"blocks\": %d, \"op\": \"%s\", \"tops\": %.3f}\n", blocks, names[i], r[i]);
  }
  hipFree(d);
  return 0;
}
