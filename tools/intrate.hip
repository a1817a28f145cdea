// Integer VALU peak-rate microbenchmark for gfx950 (P_mad of the roofline).
//
// Each lane runs 8 independent v_mad_u64_u32 chains written in inline asm
// (so the compiler cannot fold or move them); the kernel is launched with
// enough waves to fill every SIMD. Prints JSON lines: Tops = lane-ops/s.
//
// Build: hipcc --offload-arch=gfx950 -O3 tools/intrate.hip -o tools/intrate
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define ITERS 2048

__global__ __launch_bounds__(256) void k_mad(uint64_t* out, uint32_t seed) {
  uint32_t a = seed ^ threadIdx.x, b = seed * 2654435761u + blockIdx.x;
  uint64_t c0 = a, c1 = b, c2 = a + 1, c3 = b + 1, c4 = a + 2, c5 = b + 2, c6 = a + 3, c7 = b + 3;
  for (int it = 0; it < ITERS; it++) {
    asm volatile(
        "v_mad_u64_u32 %0, s[100:101], %8, %9, %0\n\t"
        "v_mad_u64_u32 %1, s[100:101], %8, %9, %1\n\t"
        "v_mad_u64_u32 %2, s[100:101], %8, %9, %2\n\t"
        "v_mad_u64_u32 %3, s[100:101], %8, %9, %3\n\t"
        "v_mad_u64_u32 %4, s[100:101], %8, %9, %4\n\t"
        "v_mad_u64_u32 %5, s[100:101], %8, %9, %5\n\t"
        "v_mad_u64_u32 %6, s[100:101], %8, %9, %6\n\t"
        "v_mad_u64_u32 %7, s[100:101], %8, %9, %7\n\t"
        : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(c4), "+v"(c5), "+v"(c6), "+v"(c7)
        : "v"(a), "v"(b)
        : "s100", "s101");
  }
  uint64_t s = c0 ^ c1 ^ c2 ^ c3 ^ c4 ^ c5 ^ c6 ^ c7;
  if (s == 0x12345) out[0] = s;
}

__global__ __launch_bounds__(256) void k_add(uint64_t* out, uint32_t seed) {
  uint32_t a = seed ^ threadIdx.x, b = seed * 2654435761u + blockIdx.x;
  uint32_t c0 = a, c1 = b, c2 = a + 1, c3 = b + 1, c4 = a + 2, c5 = b + 2, c6 = a + 3, c7 = b + 3;
  for (int it = 0; it < ITERS; it++) {
    asm volatile(
        "v_add_u32 %0, %8, %0\n\t"
        "v_add_u32 %1, %8, %1\n\t"
        "v_add_u32 %2, %8, %2\n\t"
        "v_add_u32 %3, %8, %3\n\t"
        "v_add_u32 %4, %8, %4\n\t"
        "v_add_u32 %5, %8, %5\n\t"
        "v_add_u32 %6, %8, %6\n\t"
        "v_add_u32 %7, %8, %7\n\t"
        : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(c4), "+v"(c5), "+v"(c6), "+v"(c7)
        : "v"(a), "v"(b));
  }
  uint64_t s = c0 ^ c1 ^ c2 ^ c3 ^ c4 ^ c5 ^ c6 ^ c7;
  if (s == 0x12345) out[0] = s;
}

#define CHAIN8(INSN)                                                                           \
  asm volatile(INSN " %0, %8, %0\n\t" INSN " %1, %8, %1\n\t" INSN " %2, %8, %2\n\t" INSN        \
                    " %3, %8, %3\n\t" INSN " %4, %8, %4\n\t" INSN " %5, %8, %5\n\t" INSN          \
                    " %6, %8, %6\n\t" INSN " %7, %8, %7\n\t"                                       \
               : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(c4), "+v"(c5), "+v"(c6), "+v"(c7) \
               : "v"(a))

#define K32(NAME, INSN)                                                                 \
  __global__ __launch_bounds__(256) void NAME(uint64_t* out, uint32_t seed) {           \
    uint32_t a = seed ^ threadIdx.x, b = seed * 2654435761u + blockIdx.x;               \
    uint32_t c0 = a, c1 = b, c2 = a + 1, c3 = b + 1, c4 = a + 2, c5 = b + 2, c6 = a + 3, \
             c7 = b + 3;                                                                \
    for (int it = 0; it < ITERS; it++) CHAIN8(INSN);                                    \
    uint64_t s = c0 ^ c1 ^ c2 ^ c3 ^ c4 ^ c5 ^ c6 ^ c7;                                 \
    if (s == 0x12345) out[0] = s;                                                       \
  }
K32(k_mul_lo, "v_mul_lo_u32")
K32(k_mul_hi, "v_mul_hi_u32")
K32(k_and, "v_and_b32")
K32(k_sub, "v_sub_u32")

// 64-bit-result ops: 8 independent 64-bit chains
#define K64(NAME, BODY)                                                                        \
  __global__ __launch_bounds__(256) void NAME(uint64_t* out, uint32_t seed) {                  \
    uint32_t a = seed ^ threadIdx.x;                                                           \
    uint64_t c0 = a, c1 = a + 1, c2 = a + 2, c3 = a + 3, c4 = a + 4, c5 = a + 5, c6 = a + 6,    \
             c7 = a + 7;                                                                       \
    for (int it = 0; it < ITERS; it++) {                                                       \
      asm volatile(BODY : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(c4), "+v"(c5), "+v"(c6), \
                   "+v"(c7) : "v"(a));                                                         \
    }                                                                                          \
    uint64_t s = c0 ^ c1 ^ c2 ^ c3 ^ c4 ^ c5 ^ c6 ^ c7;                                        \
    if (s == 0x12345) out[0] = s;                                                              \
  }
#define B8(I) I(0) I(1) I(2) I(3) I(4) I(5) I(6) I(7)
#define LSHLADD(n) "v_lshl_add_u64 %" #n ", %" #n ", 1, %" #n "\n\t"
#define LSHR64(n) "v_lshrrev_b64 %" #n ", 3, %" #n "\n\t"
#define MADU24(n) "v_mad_u32_u24 %" #n ", %8, %8, %" #n "\n\t"
K64(k_lshl_add_u64, B8(LSHLADD))
K64(k_lshr_b64, B8(LSHR64))
__global__ __launch_bounds__(256) void k_mad_u24(uint64_t* out, uint32_t seed) {
  uint32_t a = seed ^ threadIdx.x, b = seed * 2654435761u + blockIdx.x;
  uint32_t c0 = a, c1 = b, c2 = a + 1, c3 = b + 1, c4 = a + 2, c5 = b + 2, c6 = a + 3, c7 = b + 3;
  for (int it = 0; it < ITERS; it++)
    asm volatile(B8(MADU24) : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(c4), "+v"(c5), "+v"(c6), "+v"(c7)
                 : "v"(a));
  uint64_t s = c0 ^ c1 ^ c2 ^ c3 ^ c4 ^ c5 ^ c6 ^ c7;
  if (s == 0x12345) out[0] = s;
}
K32(k_mul_u24, "v_mul_u32_u24")
K32(k_lshl, "v_lshlrev_b32")

template <typename K>
double run(K kern, int blocks, uint64_t* d) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  kern<<<blocks, 256>>>(d, 7);
  (void)hipDeviceSynchronize();
  const int R = 5;
  (void)hipEventRecord(e0);
  for (int r = 0; r < R; r++) kern<<<blocks, 256>>>(d, 7 + r);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  double ops = (double)R * blocks * 256.0 * ITERS * 8;
  return ops / (ms * 1e-3) / 1e12;
}

int main() {
  uint64_t* d;
  (void)hipMalloc(&d, 64);
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  for (int per_cu : {1, 2, 4, 8}) {
    int blocks = cus * per_cu;  // 256-thread blocks: per_cu waves per SIMD
    printf("{\"op\": \"v_mad_u64_u32\", \"waves_per_simd\": %d, \"tops\": %.3f}\n", per_cu, run(k_mad, blocks, d));
    printf("{\"op\": \"v_add_u32\", \"waves_per_simd\": %d, \"tops\": %.3f}\n", per_cu, run(k_add, blocks, d));
    printf("{\"op\": \"v_mul_lo_u32\", \"waves_per_simd\": %d, \"tops\": %.3f}\n", per_cu, run(k_mul_lo, blocks, d));
    printf("{\"op\": \"v_mul_u32_u24\", \"waves_per_simd\": %d, \"tops\": %.3f}\n", per_cu, run(k_mul_u24, blocks, d));
    printf("{\"op\": \"v_lshlrev_b32\", \"waves_per_simd\": %d, \"tops\": %.3f}\n", per_cu, run(k_lshl, blocks, d));
    printf("{\"op\": \"v_mul_hi_u32\", \"waves_per_simd\": %d, \"tops\": %.3f}\n", per_cu, run(k_mul_hi, blocks, d));
    printf("{\"op\": \"v_and_b32\", \"waves_per_simd\": %d, \"tops\": %.3f}\n", per_cu, run(k_and, blocks, d));
    printf("{\"op\": \"v_sub_u32\", \"waves_per_simd\": %d, \"tops\": %.3f}\n", per_cu, run(k_sub, blocks, d));
    printf("{\"op\": \"v_lshl_add_u64\", \"waves_per_simd\": %d, \"tops\": %.3f}\n", per_cu, run(k_lshl_add_u64, blocks, d));
    printf("{\"op\": \"v_lshrrev_b64\", \"waves_per_simd\": %d, \"tops\": %.3f}\n", per_cu, run(k_lshr_b64, blocks, d));
    printf("{\"op\": \"v_mad_u32_u24\", \"waves_per_simd\": %d, \"tops\": %.3f}\n", per_cu, run(k_mad_u24, blocks, d));
  }
  (void)hipFree(d);
  return 0;
}
