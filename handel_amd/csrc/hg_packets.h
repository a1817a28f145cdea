// hg_packets.h — Handel packet intake on the device (hg_packets.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/handel_gpu.h"

namespace hg {

// ceil(log2(size)) (utils.go:8-11 log2)
__host__ __device__ inline int pkt_log2_ceil(uint64_t size) {
  int r = 0;
  while (r < 40 && (1ull << r) < size) r++;
  return r;
}

// binomialPartitioner.rangeLevel (partitioner.go:133-178) of node `id` in a
// registry of `size`: [lo, hi) at `level`; false for an out-of-bound level or
// an empty range (errEmptyLevel)
__host__ __device__ inline bool pkt_range_level(uint32_t id, uint32_t size, int level, uint32_t& lo, uint32_t& hi) {
  const int bitsize = pkt_log2_ceil(size);
  if (level < 0 || level > bitsize + 1) return false;
  uint64_t l = 0, h = 1ull << bitsize;
  const int inverse_idx = level - 1;
  for (int idx = bitsize - 1; idx >= inverse_idx && idx >= 0 && l < h; idx--) {
    const uint64_t middle = (h + l) / 2;
    const bool bit = (id >> idx) & 1u;
    if (bit == (idx == inverse_idx)) h = middle;
    else l = middle;
  }
  if (l >= size) return false;
  lo = (uint32_t)l;
  hi = (uint32_t)(h < size ? h : size);
  return true;
}

// words per request slot: the largest level holds 2^(ceil(log2 N) - 1) ids
inline size_t pkt_stride_words(uint64_t nreg) {
  const int b = pkt_log2_ceil(nreg);
  const uint64_t top = b > 0 ? 1ull << (b - 1) : 1;
  return (size_t)((top + 63) / 64);
}

// hg_parse_packets' kernel: slot i / n + i outputs as include/handel_gpu.h
// documents; `stride` words per request slot
void launch_parse_packets(const uint8_t* pool, uint64_t pool_len, const hg_packet* pkts, int n, uint32_t nreg,
                          int flavor, int stride, hg_request* reqs, uint64_t* words, uint8_t* sigs, int32_t* codes,
                          hipStream_t s);

}  // namespace hg
