// hg_packets.hip — Handel packet intake on the device: the parse step of
// Handel.NewPacket (handel.go:127-152) for a batch of received packets, turned
// straight into the verification requests of processing.go's verifySignature.
//
// One wave per packet. The wire parse is a handful of wave-uniform header reads
// (every lane computes the same values, no divergence); the lanes then split the
// bitset words (the empty-bitset scan, the masked copy into the request's word
// slot) and the signature bytes. Per packet the work is ~ the packet's bytes in
// and its request slot out: HBM/latency bound, no arithmetic to speak of except
// the signature's on-curve check (the same decode the verification path uses).
#include "hg_packets.h"

#include "bn256_decode.h"

namespace hg {

namespace {

HG_DEV uint32_t be16(const uint8_t* p) { return ((uint32_t)p[0] << 8) | p[1]; }
HG_DEV uint64_t be64(const uint8_t* p) {
  uint64_t v = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) v = (v << 8) | p[k];
  return v;
}

// SigBLS.UnmarshalBinary on a byte range (bn256/go/bn256.go:182-190: x/crypto
// G1.Unmarshal wants exactly 64 bytes; bn256/cf/bn256.go:183-190: cloudflare
// wants at least 64 and ignores the rest), then the point rules of decode_g1_one
HG_DEV int32_t sig_unmarshal(const uint8_t* m, uint32_t len, int flavor) {
  if (flavor == HG_FLAVOR_GO && len != 64) return HG_ERR_SIG_UNMARSHAL;
  if (flavor == HG_FLAVOR_CF && len < 64) return HG_ERR_SIG_CF_SHORT;
  PointG1 P;
  return decode_g1_one(m, flavor, P);
}

// binary.Read of `want` bytes from a reader holding `avail`: io.ReadFull's
// EOF (nothing read) / ErrUnexpectedEOF (a partial read)
HG_DEV int32_t short_read(uint64_t avail) { return avail == 0 ? HG_ERR_PKT_EOF : HG_ERR_PKT_UNEXPECTED_EOF; }

}  // namespace

__global__ __launch_bounds__(256) void k_parse_packets(const uint8_t* pool, uint64_t pool_len, const hg_packet* pkts,
                                                       int n, uint32_t nreg, int flavor, int stride, hg_request* reqs,
                                                       uint64_t* words, uint8_t* sigs, int32_t* codes) {
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= n) return;  // wave-uniform
  const hg_packet P = pkts[i];
  int32_t code = HG_OK;
  // the pool ranges (API contract; checked so a bad one never reads outside)
  const bool has_ind = (P.flags & HG_PKT_HAS_IND) != 0;
  if ((uint64_t)P.ms_off + P.ms_len > pool_len || (has_ind && (uint64_t)P.ind_off + P.ind_len > pool_len) ||
      P.receiver >= nreg)
    code = HG_ERR_ARG;
  // validatePacket (handel.go:371-385): origin, then the level among the
  // receiver's levels (createLevels: Partitioner.Levels = 1..MaxLevel, non-empty)
  uint32_t lo = 0, hi = 0;
  if (code == HG_OK && (P.origin < 0 || (uint32_t)P.origin >= nreg)) code = HG_ERR_PKT_ORIGIN;
  if (code == HG_OK &&
      !(P.level >= 1 && (int)P.level <= pkt_log2_ceil(nreg) && pkt_range_level(P.receiver, nreg, (int)P.level, lo, hi)))
    code = HG_ERR_PKT_LEVEL;
  // MultiSignature.Unmarshal (crypto.go:86-110)
  const uint8_t* m = pool + P.ms_off;
  const uint32_t L = P.ms_len;
  uint32_t blob_len = 0, wl = 0;
  uint64_t flen = 0, nwords = 0;
  if (code == HG_OK) {
    if (L < 2) code = short_read(L);  // the u16 blob length
    else {
      blob_len = be16(m);
      if (L - 2 < blob_len) code = HG_ERR_PKT_BITSET_SHORT;
    }
  }
  const uint8_t* blob = m + 2;
  if (code == HG_OK) {
    // WilffBitSet.UnmarshalBinary (bitset.go:166-177): u16 bit length, then
    // willf ReadFrom: u64 length, New(length), binary.Read of its words
    if (blob_len < 2) code = short_read(blob_len);
    else if (blob_len - 2 < 8) {
      wl = be16(blob);
      code = short_read(blob_len - 2);
    } else {
      wl = be16(blob);
      flen = be64(blob + 2);
      // wordsNeeded (capped at Cap() >> 6); make() of more than 2^48 bytes
      // panics inside New, which recovers to an empty set: length mismatch
      const uint64_t need = flen > ~0ull - 63 ? (~0ull >> 6) : (flen + 63) >> 6;
      const uint64_t avail = blob_len - 10;
      if (need > (1ull << 45)) code = HG_ERR_PKT_TYPE_MISMATCH;
      else if (need > 0 && avail < need * 8) code = short_read(avail);
      else nwords = need;
    }
  }
  const uint32_t sig_at = 2 + blob_len;
  if (code == HG_OK) code = sig_unmarshal(m + sig_at, L - sig_at, flavor);
  // parseSignatures (handel.go:389-436)
  if (code == HG_OK && wl != hi - lo) code = HG_ERR_PKT_BITSET_SIZE;
  if (code == HG_OK) {
    // m.None(): willf's whole words, bits past either length included
    bool any = false;
    for (uint64_t j = lane; j < nwords; j += 64) any |= be64(blob + 10 + 8 * j) != 0;
    if (__ballot(any) == 0) code = HG_ERR_PKT_NO_SIG;
  }
  int32_t ind_code = has_ind ? HG_OK : HG_PKT_NO_IND;
  if (code == HG_OK && has_ind) {
    code = sig_unmarshal(pool + P.ind_off, P.ind_len, flavor);
    // IndexAtLevel(origin, level): the origin inside the receiver's range
    if (code == HG_OK && ((uint32_t)P.origin < lo || (uint32_t)P.origin >= hi)) code = HG_ERR_PKT_ID_RANGE;
  }
  if (code != HG_OK) ind_code = code;

  // outputs: slot i (multisignature) and slot n + i (individual signature)
  const uint64_t lim = flen < wl ? flen : wl;  // BitSet.Get(i): i < w.l and i < willf length
  uint64_t* w1 = words + (size_t)i * stride;
  uint64_t* w2 = words + ((size_t)n + i) * stride;
  const uint32_t bit = code == HG_OK && has_ind ? (uint32_t)P.origin - lo : ~0u;
  for (int j = lane; j < stride; j += 64) {
    uint64_t v = 0;
    if (code == HG_OK && (uint64_t)j < nwords && 64ull * j < lim) {
      v = be64(blob + 10 + 8 * (size_t)j);
      const uint64_t rem = lim - 64ull * j;
      if (rem < 64) v &= (1ull << rem) - 1;
    }
    w1[j] = v;
    w2[j] = (bit >> 6) == (uint32_t)j ? 1ull << (bit & 63) : 0ull;
  }
  const bool sig_ok = code == HG_OK;
  sigs[(size_t)i * 64 + lane] = sig_ok ? m[sig_at + lane] : 0;
  sigs[((size_t)n + i) * 64 + lane] = sig_ok && has_ind ? pool[P.ind_off + lane] : 0;
  if (lane == 0) {
    const uint32_t size = hi - lo;
    reqs[i] = hg_request{lo, wl, size, (uint32_t)((size_t)i * stride)};
    reqs[n + i] = hg_request{lo, size, size, (uint32_t)(((size_t)n + i) * stride)};
    codes[i] = code;
    codes[n + i] = ind_code;
  }
}

void launch_parse_packets(const uint8_t* pool, uint64_t pool_len, const hg_packet* pkts, int n, uint32_t nreg,
                          int flavor, int stride, hg_request* reqs, uint64_t* words, uint8_t* sigs, int32_t* codes,
                          hipStream_t s) {
  if (n > 0)
    k_parse_packets<<<(n + 3) / 4, 256, 0, s>>>(pool, pool_len, pkts, n, nreg, flavor, stride, reqs, words, sigs,
                                                codes);
}

}  // namespace hg
