// bn256_agg.h — the per-request aggregation plan shared by the G2 fold
// (bn256_kernels.hip: k_agg_plan, k_aggregate, k_agg_finish) and the GT fold
// (bn256_gt.hip): bitset words in registry-aligned windows, set and nonzero
// window-byte counts, and the block-complement decision.
#pragma once
#include "bn256_kernels.h"

namespace hg {

// The per-request plan shared by the ordering and the fold kernels: set count,
// whether the block complement applies (and at which level), table points to
// fold m (nonzero bytes of the folded mask in registry-aligned windows), and
// the lanes L that fold them.
struct AggPlan {
  uint32_t cnt, m;
  int k, lanes;
  bool comp;
};
HG_DEV uint64_t agg_word(const AggRequest& q, const uint64_t* words, uint32_t wi) {
  uint64_t w = words[q.word_offset + wi];
  const uint32_t lo = wi * 64;
  if (lo + 64 > q.bitlen) w &= (1ull << (q.bitlen - lo)) - 1;
  return w;
}
// request word wi of the folded mask (complemented within bitlen when comp); 0 outside
HG_DEV uint64_t agg_mask_word(const AggRequest& q, const uint64_t* words, int wi, bool comp) {
  const int nw = (int)((q.bitlen + 63) / 64);
  if (wi < 0 || wi >= nw) return 0;
  uint64_t w = words[q.word_offset + wi];
  if (comp) w = ~w;
  const uint32_t lo = (uint32_t)wi * 64;
  if (lo + 64 > q.bitlen) w &= (1ull << (q.bitlen - lo)) - 1;
  return w;
}
// registry-aligned word v of the mask: bit j = registry slot (offset & ~7) + 64 v + j
HG_DEV uint64_t agg_rword(const AggRequest& q, const uint64_t* words, int v, bool comp) {
  const int sh = (int)(q.offset & 7u);
  const uint64_t hi = agg_mask_word(q, words, v, comp);
  if (sh == 0) return hi;
  return (hi << sh) | (agg_mask_word(q, words, v - 1, comp) >> (64 - sh));
}
HG_DEV uint32_t agg_nrwords(const AggRequest& q) { return (q.bitlen + (q.offset & 7u) + 63) / 64; }
HG_DEV uint32_t nz_bytes(uint64_t x) {
  x |= x >> 4;
  x |= x >> 2;
  x |= x >> 1;
  return __popcll(x & 0x0101010101010101ull);
}
// The same for registry-aligned windows of W bits (W = 8: the byte windows
// above; W = 16: the GT fold's 16-key windows, bn256_gt.hip)
template <int W>
HG_DEV uint64_t agg_rword_w(const AggRequest& q, const uint64_t* words, int v, bool comp) {
  const int sh = (int)(q.offset & (uint32_t)(W - 1));
  const uint64_t hi = agg_mask_word(q, words, v, comp);
  if (sh == 0) return hi;
  return (hi << sh) | (agg_mask_word(q, words, v - 1, comp) >> (64 - sh));
}
template <int W>
HG_DEV uint32_t agg_nrwords_w(const AggRequest& q) {
  return (q.bitlen + (q.offset & (uint32_t)(W - 1)) + 63) / 64;
}
HG_DEV uint32_t nz_halves(uint64_t x) {  // nonzero 16-bit quarters of x
  x |= x >> 8;
  x |= x >> 4;
  x |= x >> 2;
  x |= x >> 1;
  return __popcll(x & 0x0001000100010001ull);
}
HG_DEV AggPlan agg_plan(const AggRequest& q, uint32_t cnt, uint32_t nz_set, uint32_t nz_unset, int nreg, int levels) {
  AggPlan p;
  p.cnt = cnt;
  const uint32_t bitlen = q.bitlen;
  int k = 0;
  while (k < 31 && (1u << k) < bitlen) k++;
  const bool aligned = bitlen > 0 && k <= levels && (q.offset & ((1u << k) - 1)) == 0 &&
                       (bitlen == (1u << k) || q.offset + bitlen == (uint32_t)nreg);
  p.k = k;
  p.comp = aligned && k > 0 && nz_unset < nz_set;
  p.m = p.comp ? nz_unset : nz_set;
  int L = 1;
  while (L < 64 && 2u * (uint32_t)(2 * L) <= p.m + 1) L *= 2;  // L ~ m / 2, power of two
  p.lanes = L;
  return p;
}


}  // namespace hg
