// bn256_verify.hip — k_verify: the batched pairing check
// e(H, pk) * e(-sig, G2Base) == 1 (PublicKey.VerifySignature, bn256/go/bn256.go:82-94),
// one 16-lane team per check, TEAMS teams per single-wave workgroup.
#define HG_DIAG_TU 1
#include <cstdlib>
#include <hip/hip_runtime.h>

#include "bn256_gt.h"
#include "bn256_pairing.h"

namespace hg {
static inline int nblk(int n, int b) { return (n + b - 1) / b; }

#ifdef HG_DIAG
__device__ uint64_t g_diag[4096 * 16];
#endif


// the Miller loop's per-check inputs (pk and sig decoded by k_decode_checks)
HG_DEV CheckCtx check_ctx(const CheckIn& I, const PointG1* hpt) {
  CheckCtx C;
  C.qx = I.pk.x;
  C.qy = I.pk.y;
  C.hx = hpt->x;
  C.hy = hpt->y;
  C.sx = I.sig.x;
  C.sy = I.sig.y;
  C.use_q = I.pk.inf == 0;
  C.use_s = I.sig.inf == 0;
  if (!C.use_q) {  // keep the (unused) doubling chain well-defined
    const Fp2 gx = HG_G2X, gy = HG_G2Y;
    C.qx = gx;
    C.qy = gy;
  }
  return C;
}

// TEAMS checks per workgroup of 16 * TEAMS lanes (one wave; LDS sized to TEAMS)
template <int TEAMS>
__global__ __launch_bounds__(64) void k_verify(const CheckIn* in, int n, const LineCoef* tab,
                                               const PointG1* hpt, int32_t* codes) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[TEAMS * kTeamWords];
  Team T = make_team(lds, kTeamWords);
  uint32_t* F = team_regs(T);
  int idx = blockIdx.x * TEAMS + (threadIdx.x >> 4);
  bool valid = idx < n;
  int ci = valid ? idx : n - 1;
  const CheckIn& I = in[ci];
  const CheckCtx C = check_ctx(I, hpt);
#ifdef HG_DIAG
  if (threadIdx.x < 16) hg_diag_acc[threadIdx.x] = 0;
  __syncthreads();
  uint64_t diag_start = __builtin_amdgcn_s_memtime();
#endif
  XStream S = x_stream();
  team_miller_check(T, F, C, tab, true, S, final_exp_hint());
#ifdef HG_DIAG
  uint64_t diag_mid = __builtin_amdgcn_s_memtime();
#endif
  team_final_exp_fc(T, F, S);  // FE^m == 1 <=> FE == 1
  bool ok = t12_is_one(T, S_F);
  if (valid && T.tl == 0 && codes[idx] == HG_OK) codes[idx] = ok ? HG_OK : HG_ERR_SIG_INVALID;
#ifdef HG_DIAG
  uint64_t diag_end = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0 && blockIdx.x < 4096) {
    for (int k = 0; k < 8; k++) g_diag[blockIdx.x * 16 + k] = hg_diag_acc[k];
    g_diag[blockIdx.x * 16 + 8] = diag_mid - diag_start;
    g_diag[blockIdx.x * 16 + 9] = diag_end - diag_mid;
    g_diag[blockIdx.x * 16 + 10] = diag_end - diag_start;
  }
#endif
}


// ---------------------------------------------------------------- split form (r06)
// The same check in two halves, for batches in flight: k_verify_ml runs the
// Miller loop alone on layout V (tools/gen_g2_schedule.py: f, its programs'
// 50 pre-pass values, the register file — 128 elements, 20480 bytes per
// 4-team wave where k_verify's 212-element region takes 33.6 KB, so a CU's
// 160 KiB holds eight waves, two per SIMD, instead of four) and stores f; the final exponentiation runs on five
// 12-lane teams per wave with the norm inversions batched (launch_fe12,
// bn256_sig12.hip); k_fe_verdicts tests FE == 1. Values, and verdicts, are
// k_verify's: the same programs in the same order, and the FE chain is
// k_verify's (Fuentes-Castaneda, bn256_sigfe.h).
template <int TEAMS>
__global__ __launch_bounds__(64) void k_verify_ml(const CheckIn* in, int n, const LineCoef* tab,
                                                  const PointG1* hpt, Gt* fe) {
  constexpr int kWords = kVTeamElems * 10;
  __shared__ __attribute__((aligned(16))) uint32_t lds[TEAMS * kWords];
  Team T = make_team(lds, kWords);
  uint32_t* F = T.base + kVRegBase * 10;
  const int idx = blockIdx.x * TEAMS + (threadIdx.x >> 4);
  const bool valid = idx < n;
  const int ci = valid ? idx : n - 1;
  const CheckIn& I = in[ci];
  const CheckCtx C = check_ctx(I, hpt);
  XStream S = x_stream();
  team_miller_check<MillerV>(T, F, C, tab, true, S, xh_none());
  Fp v;
  ld_fp(v, slot(T, S_F) + T.e * 10);
  if (valid && T.active) {
    uint2* dst = (uint2*)__builtin_assume_aligned(fe[idx].w + 10 * T.e, 8);
#pragma unroll
    for (int i = 0; i < 5; i++) dst[i] = make_uint2(v.l[2 * i], v.l[2 * i + 1]);
  }
}

// codes[c] = FE(f_c) == 1 ? HG_OK : HG_ERR_SIG_INVALID where still HG_OK
// (k_verify's t12_is_one: element 1 = c0.y is one, every other element zero)
__global__ __launch_bounds__(256) void k_fe_verdicts(const Gt* fe, int n, int32_t* codes) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= n || codes[c] != HG_OK) return;
  Fp one;
  fp_one(one);
  uint32_t diff = 0;
  for (int e = 0; e < 12; e++)
#pragma unroll
    for (int l = 0; l < 10; l++) diff |= fe[c].w[10 * e + l] ^ (e == 1 ? one.l[l] : 0u);
  codes[c] = diff == 0 ? HG_OK : HG_ERR_SIG_INVALID;
}

size_t verify_split_ws_bytes(int n) { return ((size_t)n * sizeof(Gt) + 255) / 256 * 256 + fe12_ws_bytes(n); }

void launch_verify_split(const CheckIn* in, int n, const LineCoef* tab, const PointG1* h, int32_t* codes,
                         uint8_t* ws, hipStream_t s) {
  if (n <= 0 || n > kSig12MaxN) return;
  Gt* fe = (Gt*)ws;
  k_verify_ml<4><<<nblk(n, 4), 64, 0, s>>>(in, n, tab, h, fe);
  launch_fe12(fe, n, ws + ((size_t)n * sizeof(Gt) + 255) / 256 * 256, s);
  k_fe_verdicts<<<nblk(n, 256), 256, 0, s>>>(fe, n, codes);
}

void launch_verify(const CheckIn* in, int n, const LineCoef* tab, const PointG1* h, int32_t* codes, hipStream_t s) {
  // HG_TEAMS_PER_BLOCK (diagnostic): fewer checks per wave -> more waves per SIMD
  static const int tpb = [] {
    const char* e = getenv("HG_TEAMS_PER_BLOCK");
    int v = e ? atoi(e) : kTeamsPerBlock;
    return (v >= 1 && v <= kTeamsPerBlock) ? v : kTeamsPerBlock;
  }();
  if (n <= 0) return;
  if (tpb == 4) k_verify<4><<<nblk(n, 4), 64, 0, s>>>(in, n, tab, h, codes);
  else if (tpb == 2) k_verify<2><<<nblk(n, 2), 32, 0, s>>>(in, n, tab, h, codes);
  else k_verify<1><<<n, 16, 0, s>>>(in, n, tab, h, codes);
}
int diag_read(uint64_t* out, size_t n) {
#ifdef HG_DIAG
  if (n > 4096 * 16) n = 4096 * 16;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_diag), n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : 1;
#else
  (void)out;
  (void)n;
  return -1;
#endif
}
}  // namespace hg
