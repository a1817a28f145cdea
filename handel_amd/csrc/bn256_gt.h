// bn256_gt.h — data of the GT aggregate-verification path (bn256_gt.hip).
#pragma once
#include "bn256_kernels.h"

namespace hg {

// An Fp12 (GT) value in HBM, in the team slot layout: element e (10 limbs of
// 26 bits, Montgomery form) at w[10 e], element order of bn256_team.h.
struct Gt {
  uint32_t w[120];
};
static constexpr int kGtChunk = 8;  // default window-table values per fold chunk (one team)
static constexpr int kGtChunkTeams = 5;  // k_gt_chunks: chunks per workgroup (five 12-lane teams)
// The fold's windows: aligned 8-key windows (256 subset products each, 61 MB
// for a 4000-key registry) or 16-key windows (65536 each, 7.9 GB, built from
// the 8-key tables): GtWork.win_bits

// per-request fold plan (k_gt_plan, k_gt_scan)
struct GtReq {
  int m;          // window-table terms of the folded mask
  int chunks;     // ceil(m / chunk)
  int comp;       // folded over the complement inside the aligned block of level k
  int k;
  int term_off;   // first term in the batch's term list
  int chunk_off;  // first chunk in the batch's chunk list
};
struct alignas(8) GtHdr {
  int terms, chunks;  // one 64-bit atomic in k_gt_plan
  int big, mid;       // requests k_gt_combine finishes: > 4 chunks / 2..4 chunks (one 64-bit atomic)
  int nlong, nshort;  // chunks of more / at most half the chunk size in k_gt_chunks' order (one 64-bit atomic)
};
// level k >= 4 block j of the registry at blk[base[k] + j] (levels <= 3 are
// entries of the window table in use)
struct GtBlockIndex {
  int base[24];
};
// device workspaces of one fold launch
struct GtWork {
  GtReq* plan;
  GtHdr* hdr;
  uint32_t* terms;
  int2* ord;       // k_gt_chunks' order: (chunk, request), long chunks from 0, short ones down from cap - 1
  int cap;         // entries of ord and partial
  Gt* partial;
  int* multi;      // 2n: the big requests from 0, the mid ones from n (k_gt_combine's order)
  int chunk_grid;  // workgroups of k_gt_chunks (one wave: kGtChunkTeams teams)
  int chunk;       // terms per chunk
  int win_bits;    // 8 or 16: which window table `win` is
};

// G_i = e(H, pk_i) for the n registry keys
void launch_gt_keys(const PointG2* reg, int n, const LineCoef* tab, const PointG1* h, Gt* out, hipStream_t s);
// w8[256 w + s] = product of G_{8w + j} over the bits j of s (absent keys = 1)
void launch_gt_windows8(const Gt* key, int nreg, Gt* w8, int nwin8, hipStream_t s);
// w16[65536 w + s] = product of G_{16w + j} over the bits j of s, from w8
void launch_gt_windows16(const Gt* w8, int nwin8, Gt* w16, int nwin16, hipStream_t s);
// dst[j] = src[2j] * src[2j + 1] (entries `stride` apart; a missing odd entry = 1)
void launch_gt_blocks(const Gt* src, int stride, int nsrc, Gt* dst, int ndst, hipStream_t s);
// the fold of n requests: y[r] = conj(e(H, aggregate key of r)); codes: level
// codes in, HG_ERR_EMPTY_AGG added for empty bitsets; zero_hdr: clear the
// range counters first (false: the caller's prologue did)
void launch_gt_fold(const AggRequest* reqs, int n, const uint64_t* words, int32_t* codes, int nreg, int levels,
                    const Gt* win, const Gt* blk, const GtBlockIndex& bi, GtWork w, Gt* y, bool zero_hdr,
                    hipStream_t s);
// FE(Miller(G2Base at -sig_r)) == y[r] for every request still HG_OK
void launch_verify_sig(const PointG1* sigs, int n, const LineCoef* tab, const Gt* y, int32_t* codes, hipStream_t s);
// the same check in two launches, so the fold can run beside the pairing:
// fe[r] = FE(Miller(G2Base at -sig_r)) from the 64-byte marshals (decoded in
// the kernel), then fe[r] == y[r] where still HG_OK
// k_verify_sig_split<2>: a check's team spread over two waves (the latency
// form, bn256_sigsplit.h); a padded launch_sig_pairing of n <= min(w2_max,
// 2048) checks takes it unless HG_SIG_W2=0. sig_w2_lane_max: the bound for
// lanes (HG_SIG_W2_LANE_MAX, 0)
static constexpr int kSigW2MaxN = 2048;
bool sig_w2_for(bool pad, int n, int w2_max);
int sig_w2_lane_max();
void launch_sig_pairing_w2(const uint8_t* sigs, int flavor, int n, const LineCoef* tab, Gt* fe, hipStream_t s);
void launch_sig_pairing(const uint8_t* sigs, int flavor, int n, const LineCoef* tab, Gt* fe, hipStream_t s,
                        bool pad = true, int w2_max = kSigW2MaxN);
// launch_sig_pairing on five 12-lane teams per wave (bn256_sig12.hip): the
// lines evaluated at -sig first (k_sig_lines, into ev: sig12_lines_bytes(n)),
// then k_verify_sig12; the same fe values
size_t sig12_lines_bytes(int n);
void launch_sig_pairing12(const uint8_t* sigs, int flavor, int n, const LineCoef* tab, Fp* ev, Gt* fe,
                          hipStream_t s, bool pad);
// which kernel a submission runs: the 12-lane one for unpadded launches (the
// throughput mode: batches in flight share the SIMDs, and a check costs 20 %
// fewer wave-instructions), the 16-lane padded k_verify_sig for padded ones
// (the latency mode: one wave per SIMD, where its shorter per-wave program
// and the absence of the line kernels give the lower batch latency).
// HG_SIG12=1 / 0 forces one kernel for every launch (A/B).
// n: the batch's checks; above kSig12MaxN the 12-lane path (whose line kernel
// indexes 4 n threads in int) is never taken
constexpr int kSig12MaxN = 1 << 28;
bool sig12_for(bool pad, size_t n = 0);
// the split chain's final exponentiation (k_sig12_norm, k_sig12_ninv,
// k_sig12_fe) of n Miller values in fe, in place: config 2's second half
// (launch_verify_split); ws: fe12_ws_bytes(n) bytes
size_t fe12_ws_bytes(int n);
void launch_fe12(Gt* fe, int n, uint8_t* ws, hipStream_t s);
void launch_gt_compare(const Gt* fe, const Gt* y, int n, int32_t* codes, hipStream_t s);
// the same, and the verdict bitset (ceil(n / 8) bytes, hg_pack_verdicts_device's layout)
void launch_gt_compare_bits(const Gt* fe, const Gt* y, int n, int32_t* codes, uint8_t* bits, hipStream_t s);

}  // namespace hg
