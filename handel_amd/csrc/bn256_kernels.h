// bn256_kernels.h — device data layout shared by the kernels and the host API.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/handel_gpu.h"
#include "bn256_fp.h"

namespace hg {

// Decoded points in HBM: affine, Montgomery form, explicit infinity flag.
struct PointG1 {
  Fp x, y;
  uint32_t inf;
  uint32_t pad[3];
};
struct PointG2 {
  Fp2 x, y;
  uint32_t inf;
  uint32_t pad[3];
};
// One pairing check: e(H, pk) * e(-sig, G2Base) == 1
struct CheckIn {
  PointG2 pk;
  PointG1 sig;
};
// A G2Base Miller-loop line, normalised: x/crypto's line c + b w + a w^3
// divided by its constant coefficient a (an Fp2 factor, removed by the final
// exponentiation), i.e. c' + b' w + w^3 with b' = bx * Px, c' = cy * Py
struct LineCoef {
  Fp2 bx, cy;
};
static constexpr int kNumLines = 65 + 18 + 2;  // doublings + NAF additions + 2 Frobenius lines

using AggRequest = hg_request;

void launch_decode_g2(const uint8_t* bytes, int n, int flavor, PointG2* out, int32_t* codes, hipStream_t s);
void launch_decode_g1(const uint8_t* bytes, int n, int flavor, PointG1* out, int32_t* codes, hipStream_t s);
// *count += the decoded keys reg[i] on the twist but outside G2 (n * P != inf)
void launch_g2_subgroup(const PointG2* reg, int n, int* count, hipStream_t s);
void launch_encode_g2(const PointG2* in, int n, uint8_t* out, hipStream_t s);
void launch_encode_g1(const PointG1* in, int n, uint8_t* out, hipStream_t s);
void launch_g2_mul_base(const uint8_t* scalars, int n, PointG2* out, hipStream_t s);
void launch_g1_mul(const PointG1* base, const uint8_t* scalars, int n, PointG1* out, hipStream_t s);
void launch_hash_point(const uint32_t* k, PointG1* out, hipStream_t s);
void launch_g2_lines(LineCoef* tab, hipStream_t s);
void launch_verify(const CheckIn* in, int n, const LineCoef* tab, const PointG1* h, int32_t* codes, hipStream_t s);
// the same checks in two halves (k_verify_ml on a compact team region, then
// the 12-lane final exponentiation): the form for batches in flight; ws:
// verify_split_ws_bytes(n) bytes
size_t verify_split_ws_bytes(int n);
void launch_verify_split(const CheckIn* in, int n, const LineCoef* tab, const PointG1* h, int32_t* codes,
                         uint8_t* ws, hipStream_t s);
void launch_pair(const PointG1* g1s, const PointG2* g2s, int n, const LineCoef* tab, uint8_t* gt, hipStream_t s);
// blocks/block_base: the aligned block sums of the registry (hg_registry_load);
// level k block j at blocks[block_base[k] + j] for 1 <= k <= levels
void launch_aggregate(const PointG2* wsum, int nreg, const PointG2* blocks, const int* block_base, int levels,
                      const AggRequest* reqs, int n, const uint64_t* words, int* order, void* partial_ws,
                      CheckIn* out, int32_t* codes, hipStream_t s);
size_t agg_partial_bytes();  // workspace bytes per request for launch_aggregate
size_t agg_fixed_bytes();    // plus this once
void launch_block_sums(const PointG2* src, int nsrc, PointG2* dst, int ndst, hipStream_t s);
// byte-window subset sums: wsum[256 w + s] = sum of reg[8 w + j] over the bits j of s
void launch_window_sums(const PointG2* reg, int nreg, PointG2* wsum, int nwin, hipStream_t s);
void launch_g1_combine(const PointG1* a, const PointG1* b, int n, uint8_t* out, hipStream_t s);
void launch_checks_from_points(const PointG2* pks, const PointG1* sigs, int n, CheckIn* out, hipStream_t s);
void launch_merge_codes(const int32_t* a, const int32_t* b, int n, int32_t* out, hipStream_t s);
// level check + signature decode + verdict precedence of an aggregate batch in
// one launch (pts, codes out); block 0 zeroes zero[0 .. zero_words) (<= 64)
void launch_agg_prologue(const AggRequest* reqs, int n, uint32_t nreg, const uint8_t* sigs, int flavor, PointG1* pts,
                         int32_t* codes, int* zero, int zero_words, hipStream_t s);
void launch_decode_checks(const uint8_t* pks, const uint8_t* sigs, int n, int flavor, CheckIn* out, int32_t* codes,
                          hipStream_t s);
void launch_pack_verdicts(const int32_t* codes, int n, uint8_t* bits, hipStream_t s);
void launch_sig_into_checks(const PointG1* sigs, int n, CheckIn* out, hipStream_t s);
void launch_extract_pk(const CheckIn* in, int n, PointG2* out, hipStream_t s);
int diag_read(uint64_t* out, size_t n);
void launch_g2_combine(const PointG2* a, const PointG2* b, int n, PointG2* out, hipStream_t s);
void launch_fp12_op(int op, const uint8_t* a, const uint8_t* b, int n, uint8_t* out, hipStream_t s);
void launch_fp_mul(const uint32_t* a, const uint32_t* b, int n, uint32_t* out, hipStream_t s);

}  // namespace hg
