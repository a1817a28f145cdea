// hg_api.cpp — host side of the C ABI declared in include/handel_gpu.h.
//
// Owns the HIP resources of one verification context and sequences the
// kernels of bn256_kernels.hip. Mirrors the reference's call structure:
//   Constructor / G2Base           -> hg_create (+ the G2Base line table)
//   registry PublicKey.Unmarshal   -> hg_registry_load (simul/lib/nodes.go:44-64)
//   hashedMessage                  -> hg_set_message (once per message)
//   PublicKey.VerifySignature      -> hg_verify_batch
//   processing.go verifySignature  -> hg_verify_aggregate
// Error precedence follows the order in which the reference surfaces errors:
// unmarshal (at parse time) > bitset/level check > hashedMessage EOF >
// nil-aggregate panic > pairing verdict.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "bn256_gt.h"
#include "bn256_kernels.h"
#include "hg_codes.h"
#include "hg_packets.h"

using namespace hg;

namespace {

// ------------------------------------------------------------ SHA-256 (FIPS 180-4)
const uint32_t kSha[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

inline uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

void sha256_block(uint32_t h[8], const uint8_t* b) {
  uint32_t w[64];
  for (int i = 0; i < 16; i++)
    w[i] = (uint32_t)b[4 * i] << 24 | (uint32_t)b[4 * i + 1] << 16 | (uint32_t)b[4 * i + 2] << 8 | b[4 * i + 3];
  for (int i = 16; i < 64; i++) {
    uint32_t s0 = rotr(w[i - 15], 7) ^ rotr(w[i - 15], 18) ^ (w[i - 15] >> 3);
    uint32_t s1 = rotr(w[i - 2], 17) ^ rotr(w[i - 2], 19) ^ (w[i - 2] >> 10);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  uint32_t a = h[0], bb = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
  for (int i = 0; i < 64; i++) {
    uint32_t t1 = hh + (rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25)) + ((e & f) ^ (~e & g)) + kSha[i] + w[i];
    uint32_t t2 = (rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22)) + ((a & bb) ^ (a & c) ^ (bb & c));
    hh = g;
    g = f;
    f = e;
    e = d + t1;
    d = c;
    c = bb;
    bb = a;
    a = t1 + t2;
  }
  h[0] += a; h[1] += bb; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

void sha256(const uint8_t* m, size_t len, uint8_t out[32]) {
  uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  size_t i = 0;
  for (; i + 64 <= len; i += 64) sha256_block(h, m + i);
  uint8_t tail[128] = {0};
  size_t rem = len - i;
  if (rem) memcpy(tail, m + i, rem);
  tail[rem] = 0x80;
  size_t tl = rem + 9 <= 64 ? 64 : 128;
  uint64_t bits = (uint64_t)len * 8;
  for (int k = 0; k < 8; k++) tail[tl - 1 - k] = (uint8_t)(bits >> (8 * k));
  sha256_block(h, tail);
  if (tl == 128) sha256_block(h, tail + 64);
  for (int k = 0; k < 8; k++) {
    out[4 * k] = (uint8_t)(h[k] >> 24);
    out[4 * k + 1] = (uint8_t)(h[k] >> 16);
    out[4 * k + 2] = (uint8_t)(h[k] >> 8);
    out[4 * k + 3] = (uint8_t)h[k];
  }
}

const uint32_t kOrder32[8] = {HG_ORDER32};

// crypto/rand.Int(bytes.NewBuffer(d), Order) as used by hashedMessage: the
// single 32-byte read is accepted iff 0 < int(d) < n; otherwise the next
// read hits EOF.
bool hash_scalar(const uint8_t d[32], uint32_t k[8]) {
  for (int i = 0; i < 8; i++) {
    const uint8_t* q = d + (7 - i) * 4;
    k[i] = (uint32_t)q[0] << 24 | (uint32_t)q[1] << 16 | (uint32_t)q[2] << 8 | q[3];
  }
  bool zero = true;
  for (int i = 0; i < 8; i++) zero &= k[i] == 0;
  if (zero) return false;
  for (int i = 7; i >= 0; i--) {
    if (k[i] < kOrder32[i]) return true;
    if (k[i] > kOrder32[i]) return false;
  }
  return false;  // equal to n
}

__global__ void k_fill_codes(int32_t* c, int n, int32_t from, int32_t to) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && c[i] == from) c[i] = to;
}
// final = sig decode error > level error > hash EOF > empty aggregate > (verify)
__global__ void k_agg_codes(const int32_t* sig_codes, const int32_t* lvl_codes, int hash_eof, int n, int32_t* out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int32_t c = sig_codes[i];
  if (c == HG_OK && lvl_codes[i] == HG_ERR_LEVEL) c = HG_ERR_LEVEL;
  if (c == HG_OK && hash_eof) c = HG_ERR_HASH_EOF;
  if (c == HG_OK) c = lvl_codes[i];
  out[i] = c;
}

template <typename T>
struct DevBuf {
  T* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t n) {
    if (n <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    size_t want = n < 64 ? 64 : n;
    hipError_t e = hipMalloc(&p, want * sizeof(T));
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

// Device workspaces of one in-flight submission: the context's own set (every
// hg_* entry point, ordered by the context's submission chain) and one set
// per service lane (hg_lane below), so several lanes' batches run at once
// over the same registry and GT tables.
struct Ws {
  DevBuf<PointG2> pts2;
  DevBuf<PointG1> pts1;
  DevBuf<CheckIn> checks;
  DevBuf<int32_t> codes_b, codes_c;
  DevBuf<int> order;       // aggregation schedule (k_agg_order)
  DevBuf<uint8_t> agg_ws;  // per-request fold results (k_aggregate -> k_agg_finish)
  // GT fold workspaces
  DevBuf<GtReq> gt_plan;
  DevBuf<GtHdr> gt_hdr;
  DevBuf<uint32_t> gt_terms;
  DevBuf<int2> gt_ord;
  DevBuf<int> gt_multi;
  DevBuf<Gt> gt_partial, gt_y;
  // the fold runs on a side stream beside the pairing kernel (GT path): the
  // FE values of the batch land in gt_fe, k_gt_compare joins the two
  hipStream_t side = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  DevBuf<Gt> gt_fe;
  // launch_sig_pairing12: the batch's lines evaluated at -sig; launch_verify_split
  // (config 2): the Miller values and the final exponentiation's records
  DevBuf<uint8_t> sig_lines;
  void release() {
    pts2.release();
    pts1.release();
    checks.release();
    codes_b.release();
    codes_c.release();
    order.release();
    agg_ws.release();
    gt_plan.release();
    gt_hdr.release();
    gt_terms.release();
    gt_ord.release();
    gt_multi.release();
    gt_partial.release();
    gt_y.release();
    gt_fe.release();
    sig_lines.release();
    if (side) (void)hipStreamDestroy(side);
    if (ev_fork) (void)hipEventDestroy(ev_fork);
    if (ev_join) (void)hipEventDestroy(ev_join);
    side = nullptr;
    ev_fork = ev_join = nullptr;
  }
  size_t bytes() const {
    return pts2.cap * sizeof(PointG2) + pts1.cap * sizeof(PointG1) + checks.cap * sizeof(CheckIn) +
           (codes_b.cap + codes_c.cap) * sizeof(int32_t) + order.cap * sizeof(int) + agg_ws.cap +
           gt_plan.cap * sizeof(GtReq) + gt_hdr.cap * sizeof(GtHdr) + gt_terms.cap * sizeof(uint32_t) +
           gt_ord.cap * sizeof(int2) + gt_multi.cap * sizeof(int) + (gt_partial.cap + gt_y.cap + gt_fe.cap) * sizeof(Gt) +
           sig_lines.cap;
  }
};

// The per-message part of the context: hashedMessage and the GT tables
// e(H, .) of the registry. The context keeps the current message's set and
// the previous one (hg_set_message switches between the two without a
// rebuild, so interleaved messages keep their tables).
struct TableSet {
  std::vector<uint8_t> msg;
  bool has_msg = false, hash_eof = false;
  PointG1* d_h = nullptr;
  DevBuf<Gt> gt_key, gt_w8, gt_win, gt_blk;
  int gt_level = 0;
  size_t gt_requests = 0;
};

}  // namespace

struct hg_ctx {
  int device = 0;
  int flavor = HG_FLAVOR_GO;
  hipStream_t stream = nullptr;
  std::mutex mu;
  std::string err;
  // constant tables
  LineCoef* d_lines = nullptr;
  PointG1* d_h = nullptr;
  uint32_t* d_k = nullptr;
  bool has_msg = false;
  bool hash_eof = false;
  std::vector<uint8_t> msg;  // the message d_h was hashed from (hg_*_msg cache)
  // registry (nreg > 0 only while every table below matches it)
  DevBuf<PointG2> reg;
  size_t nreg = 0;
  // aligned block sums of the registry (level k block j at blocks[block_base[k] + j])
  DevBuf<PointG2> blocks;
  // subset sums of every aligned 8-key window (256 per window), the fold's table
  DevBuf<PointG2> wsum;
  std::vector<int> block_base = std::vector<int>(24, 0);
  int block_levels = 0;
  // workspaces
  Ws ws;
  DevBuf<uint8_t> bytes_a, bytes_b;
  DevBuf<PointG1> pts1b;
  DevBuf<int32_t> codes_a;
  DevBuf<hg_request> reqs;
  DevBuf<hg_packet> pkts;  // hg_parse_packets staging
  DevBuf<uint64_t> words;
  // GT path of aggregate verification (bn256_gt.hip): e(H, pk_i), window
  // subset products and block products, valid for the current message and
  // registry (rebuilt by the first aggregate submission after either changes)
  // 0: none (aggregates use the G2 fold); 1: e(H, pk_i), 8-key windows and
  // blocks; 2: + 16-key windows. Reset by a message or registry change;
  // raised by hg_prepare_aggregate or by request volume (gt_requests).
  int gt_level = 0;
  size_t gt_requests = 0;
  // -1: the volume policy; 0..2: every aggregate submission at that level
  // (hg_set_aggregate_level; HG_GT_LEVEL / HG_AGG_PATH give the default)
  int pinned_level = -1;
  // highest level this registry may use: lowered when the device (or the
  // table budget) could not hold a level's tables, reset by a registry load
  int gt_cap = 2;
  size_t table_budget = SIZE_MAX;  // bytes of GT tables (hg_set_table_budget)
  // registry keys on the twist but outside G2 (go flavor only: x/crypto's
  // Unmarshal accepts them); any such key pins the registry to level 0. The
  // check (one n*Q per key, ~7 ms of single-lane latency) runs on the side
  // stream after the load; it is waited for only when a GT level is wanted.
  size_t reg_non_g2 = 0;
  bool sub_pending = false;
  hipEvent_t ev_sub = nullptr;
  DevBuf<int> sub_count;
  DevBuf<Gt> gt_key, gt_w8, gt_win, gt_blk;  // gt_w8: 8-key windows, gt_win: 16-key windows
  GtBlockIndex gt_bi{};
  // the previous message's hashedMessage and tables (swapped with the fields
  // above by set_message_locked; see TableSet)
  TableSet alt;
  // the cap a failed device allocation set (gt_cap also follows the table
  // budget; hg_set_table_budget re-derives gt_cap from this)
  int oom_cap = 2;
  bool overlap = true;  // hg_set_fold_overlap; HG_GT_OVERLAP=0 gives new contexts false
  bool verify_split = false;  // hg_set_verify_split; HG_VERIFY_SPLIT=1 gives new contexts true
  // submission order across streams: the event recorded after the last
  // submission and the stream it ran on (the workspaces above are shared)
  hipEvent_t last_ev = nullptr;
  hipStream_t last_s = nullptr;
  // service lanes (hg_lane): batches in flight on their own workspaces and
  // streams; every context submission first waits for their last batches
  // (they read the registry, H and the tables a submission may rewrite)
  std::vector<hg_lane*> lanes;
  // optional per-phase timing (bench roofline), see hg_timing_read_phase
  bool timing = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> events[HG_NUM_PHASES];
};

// One service lane (hg_service.cpp): one batch at a time in flight on its own
// stream and workspaces, beside the other lanes' batches. The batch's inputs
// (requests | signatures | bitset words) are staged in pinned host memory and
// go to the device in ONE copy; the codes come back the same way.
struct hg_lane {
  hg_ctx* c = nullptr;
  Ws ws;
  hipStream_t s = nullptr;
  hipEvent_t done = nullptr;
  bool recorded = false;  // `done` marks the lane's last batch
  bool overlap = true;    // the fold beside the pairing kernel (on ws.side)
  bool pad = true;        // one pairing wave per SIMD (hg_lane_set_pairing_padding)
  int w2_max = sig_w2_lane_max();  // the two-wave latency form up to this batch (hg_lane_set_latency_form)
  hipEvent_t ev_in = nullptr;  // hg_lane_submit_device: the caller's stream point
  size_t max_batch = 0, max_words = 0;
  uint8_t* h_in = nullptr;     // pinned staging
  int32_t* h_codes = nullptr;  // pinned
  DevBuf<uint8_t> d_in;
  DevBuf<int32_t> d_codes;
  size_t n = 0, nwords = 0, off_sigs = 0, off_words = 0, in_bytes = 0;
};

// ---------------------------------------------------------------- submission order
// Every device submission of a context runs between begin() and end(): a
// submission on another stream than the previous one first waits for the
// previous one's event, so two submissions never use the shared workspaces
// (or the registry tables and H) at the same time. Service lanes keep their
// own workspaces; a context submission waits for each lane's last batch.
static hipError_t begin(hg_ctx* c, hipStream_t s) {
  if (c->last_ev && c->last_s != s) {
    hipError_t e = hipStreamWaitEvent(s, c->last_ev, 0);
    if (e != hipSuccess) return e;
  }
  for (hg_lane* l : c->lanes) {
    if (!l->recorded) continue;
    hipError_t e = hipStreamWaitEvent(s, l->done, 0);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}
static hipError_t end(hg_ctx* c, hipStream_t s) {
  if (!c->last_ev) {
    hipError_t e = hipEventCreateWithFlags(&c->last_ev, hipEventDisableTiming);
    if (e != hipSuccess) return e;
  }
  c->last_s = s;
  return hipEventRecord(c->last_ev, s);
}
// One submission: end() runs on every exit once start() succeeded, error
// returns included, so a later submission on another stream still waits for
// whatever this one had queued.
struct Submission {
  hg_ctx* c;
  hipStream_t s;
  bool open = false;
  Submission(hg_ctx* c_, hipStream_t s_) : c(c_), s(s_) {}
  hipError_t start() {
    hipError_t e = begin(c, s);
    open = e == hipSuccess;
    return e;
  }
  hipError_t finish() {
    open = false;
    return end(c, s);
  }
  ~Submission() {
    if (open) (void)end(c, s);
  }
};

// ---------------------------------------------------------------- timing
struct PhaseTimer {
  hg_ctx* c;
  int phase;
  hipStream_t s;
  hipEvent_t a = nullptr, b = nullptr;
  PhaseTimer(hg_ctx* c_, int phase_, hipStream_t s_) : c(c_), phase(phase_), s(s_) {
    if (!c->timing) return;
    if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) {
      if (a) (void)hipEventDestroy(a);
      a = b = nullptr;
      return;
    }
    (void)hipEventRecord(a, s);
  }
  void stop() {
    if (!a) return;
    (void)hipEventRecord(b, s);
    c->events[phase].emplace_back(a, b);
    a = b = nullptr;
  }
  ~PhaseTimer() {  // an error path that never reached stop(): discard
    if (a) (void)hipEventDestroy(a);
    if (b) (void)hipEventDestroy(b);
  }
};

// config 2's split form (launch_verify_split: the Miller loop on a compact
// team region, the 12-lane final exponentiation): hg_set_verify_split
static bool verify_split_for(const hg_ctx* c, size_t n) { return c->verify_split && n <= (size_t)kSig12MaxN; }

static void timed_verify(hg_ctx* c, const CheckIn* in, int n, int32_t* codes, hipStream_t s,
                         uint8_t* split_ws = nullptr) {
  PhaseTimer t(c, HG_PHASE_VERIFY, s);
  if (split_ws) launch_verify_split(in, n, c->d_lines, c->d_h, codes, split_ws, s);
  else launch_verify(in, n, c->d_lines, c->d_h, codes, s);
  t.stop();
}

#define HG_CHECK(ctx, expr)                                                        \
  do {                                                                             \
    hipError_t e_ = (expr);                                                        \
    if (e_ != hipSuccess) {                                                        \
      (ctx)->err = std::string(#expr) + ": " + hipGetErrorString(e_);              \
      return HG_ERR_DEVICE;                                                        \
    }                                                                              \
  } while (0)

static int nb(size_t n) { return (int)((n + 255) / 256); }

static int check_launch(hg_ctx* c) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    c->err = std::string("kernel launch: ") + hipGetErrorString(e);
    return HG_ERR_DEVICE;
  }
  return HG_OK;
}

static void release_tables(TableSet& t) {
  t.gt_key.release();
  t.gt_w8.release();
  t.gt_win.release();
  t.gt_blk.release();
  t.gt_level = 0;
}

static void release_all(hg_ctx* c) {
  c->reg.release();
  c->blocks.release();
  c->wsum.release();
  c->bytes_a.release();
  c->bytes_b.release();
  c->pts1b.release();
  c->codes_a.release();
  c->reqs.release();
  c->words.release();
  c->gt_key.release();
  c->gt_w8.release();
  c->gt_win.release();
  c->gt_blk.release();
  c->gt_level = 0;
  release_tables(c->alt);
  if (c->alt.d_h) (void)hipFree(c->alt.d_h);
  c->alt.d_h = nullptr;
  c->alt.has_msg = false;
  c->ws.release();
  if (c->ev_sub) (void)hipEventDestroy(c->ev_sub);
  c->sub_count.release();
  c->sub_pending = false;
  c->ev_sub = nullptr;
  for (auto& ph : c->events) {
    for (auto& pr : ph) {
      (void)hipEventDestroy(pr.first);
      (void)hipEventDestroy(pr.second);
    }
    ph.clear();
  }
  if (c->last_ev) (void)hipEventDestroy(c->last_ev);
  c->last_ev = nullptr;
  if (c->d_lines) (void)hipFree(c->d_lines);
  if (c->d_h) (void)hipFree(c->d_h);
  if (c->d_k) (void)hipFree(c->d_k);
  c->d_lines = nullptr;
  c->d_h = nullptr;
  c->d_k = nullptr;
  if (c->stream) (void)hipStreamDestroy(c->stream);
  c->stream = nullptr;
}

// exchanges the context's current message part with the cached one
static void swap_tables(hg_ctx* c) {
  TableSet& t = c->alt;
  std::swap(c->msg, t.msg);
  std::swap(c->has_msg, t.has_msg);
  std::swap(c->hash_eof, t.hash_eof);
  std::swap(c->d_h, t.d_h);
  std::swap(c->gt_key, t.gt_key);
  std::swap(c->gt_w8, t.gt_w8);
  std::swap(c->gt_win, t.gt_win);
  std::swap(c->gt_blk, t.gt_blk);
  std::swap(c->gt_level, t.gt_level);
  std::swap(c->gt_requests, t.gt_requests);
}

static bool same_msg(const std::vector<uint8_t>& m, const uint8_t* msg, size_t len) {
  return m.size() == len && (len == 0 || memcmp(m.data(), msg, len) == 0);
}

// hashedMessage into d_h (the caller holds the lock); HG_OK or HG_ERR_HASH_EOF.
// The context keeps two messages (bn256/go/bn256.go:210-218: H and with it
// every GT table is fixed per message): the current one and the previous one.
// Switching back to the previous message swaps the two sets and keeps its
// tables; a third message takes over the older set's buffers (level 0, its
// tables rebuilt on demand). The hash and any later rebuild run in
// submission order, after every submission that still reads the old set.
static int set_message_locked(hg_ctx* c, const uint8_t* msg, size_t len) {
  HG_CHECK(c, hipSetDevice(c->device));
  if (c->has_msg && same_msg(c->msg, msg, len)) return c->hash_eof ? HG_ERR_HASH_EOF : HG_OK;
  if (c->alt.has_msg && same_msg(c->alt.msg, msg, len)) {
    swap_tables(c);
    return c->hash_eof ? HG_ERR_HASH_EOF : HG_OK;
  }
  // the current set becomes the cached one; the new message takes the other
  if (c->has_msg) swap_tables(c);
  if (!c->d_h) HG_CHECK(c, hipMalloc(&c->d_h, sizeof(PointG1)));
  uint8_t d[32];
  sha256(msg, len, d);
  uint32_t k[8];
  c->has_msg = false;
  c->gt_level = 0;  // these buffers hold e(H, .) of an evicted message
  c->gt_requests = 0;
  c->msg.assign(msg, msg + len);
  c->hash_eof = !hash_scalar(d, k);
  if (c->hash_eof) {
    c->has_msg = true;
    return HG_ERR_HASH_EOF;
  }
  Submission sub(c, c->stream);
  HG_CHECK(c, sub.start());
  HG_CHECK(c, hipMemcpyAsync(c->d_k, k, sizeof k, hipMemcpyHostToDevice, c->stream));
  launch_hash_point(c->d_k, c->d_h, c->stream);
  int rc = check_launch(c);
  if (rc) return rc;
  HG_CHECK(c, sub.finish());
  HG_CHECK(c, hipStreamSynchronize(c->stream));
  c->has_msg = true;
  return HG_OK;
}

static int verify_batch_device_locked(hg_ctx* c, const uint8_t* d_pks, const uint8_t* d_sigs, size_t n,
                                      int32_t* d_codes, hipStream_t s) {
  if (!c->has_msg) {
    c->err = "hg_set_message was not called";
    return HG_ERR_ARG;
  }
  HG_CHECK(c, c->ws.checks.ensure(n));
  const bool split = verify_split_for(c, n);
  if (split) HG_CHECK(c, c->ws.sig_lines.ensure(verify_split_ws_bytes((int)n)));
  Submission sub(c, s);
  HG_CHECK(c, sub.start());
  PhaseTimer all(c, HG_PHASE_SUBMIT, s);
  launch_decode_checks(d_pks, d_sigs, (int)n, c->flavor, c->ws.checks.p, d_codes, s);
  if (c->hash_eof) k_fill_codes<<<nb(n), 256, 0, s>>>(d_codes, (int)n, HG_OK, HG_ERR_HASH_EOF);
  else timed_verify(c, c->ws.checks.p, (int)n, d_codes, s, split ? c->ws.sig_lines.p : nullptr);
  all.stop();
  int rc = check_launch(c);
  if (rc) return rc;
  HG_CHECK(c, sub.finish());
  return HG_OK;
}

static int verify_batch_host_locked(hg_ctx* c, const uint8_t* pks, const uint8_t* sigs, size_t n, int32_t* codes) {
  HG_CHECK(c, hipSetDevice(c->device));
  HG_CHECK(c, c->bytes_a.ensure(n * 128));
  HG_CHECK(c, c->bytes_b.ensure(n * 64));
  HG_CHECK(c, c->ws.codes_c.ensure(n));
  Submission sub(c, c->stream);
  HG_CHECK(c, sub.start());
  HG_CHECK(c, hipMemcpyAsync(c->bytes_a.p, pks, n * 128, hipMemcpyHostToDevice, c->stream));
  HG_CHECK(c, hipMemcpyAsync(c->bytes_b.p, sigs, n * 64, hipMemcpyHostToDevice, c->stream));
  int rc = verify_batch_device_locked(c, c->bytes_a.p, c->bytes_b.p, n, c->ws.codes_c.p, c->stream);
  if (rc) return rc;
  HG_CHECK(c, hipMemcpyAsync(codes, c->ws.codes_c.p, n * 4, hipMemcpyDeviceToHost, c->stream));
  HG_CHECK(c, sub.finish());
  HG_CHECK(c, hipStreamSynchronize(c->stream));
  return HG_OK;
}

// host-side request validation: the level check of processing.go:350-352
static void level_codes(hg_ctx* c, const hg_request* reqs, size_t n, std::vector<int32_t>& out) {
  out.resize(n);
  for (size_t i = 0; i < n; i++) {
    const hg_request& r = reqs[i];
    bool ok = r.bitlen == r.level_size && (size_t)r.offset + r.bitlen <= c->nreg;
    out[i] = ok ? HG_OK : HG_ERR_LEVEL;
  }
}

// The GT tables. Level 1 (e(H, pk_i) for every key, 8-key window subset
// products, aligned block products: ≈ 3 ms and 61 MB for 4000 keys) saves
// ≈ 0.6 ms per 4096-request batch against the G2 fold (config 3), so it pays
// for itself after ≈ 20 k requests of one message; level 2 (16-key windows:
// ≈ 12.5 ms more and ≈ 1.97 MB of HBM per key, registries up to 16384 keys)
// saves another ≈ 0.05 ms per batch and pays off after ≈ 1 M requests. The
// thresholds are those break-even volumes (a rent-or-buy rule: at most about
// twice the cost of the better choice in hindsight). A message or registry
// change drops the tables and restarts the count. hg_prepare_aggregate builds
// the top level at once (serving). hg_set_aggregate_level pins a level per
// context (0 = G2 fold only); HG_GT_LEVEL=0/1/2 (HG_AGG_PATH=g2 = 0) is the
// pinned level of new contexts (tests and A/B runs).
//
// The tables are a cache, never a requirement: a level whose tables (or fold
// workspaces) the device cannot hold, or that exceeds the context's table
// budget, lowers the context's cap and the submission runs at the level below
// (down to the G2 fold, which needs no tables). A registry with a key outside
// G2 stays at level 0 (the GT product equals e(H, sum) only on G2).
static constexpr size_t kGtMaxRegistry = 16384;
static constexpr size_t kGtLevel1Requests = 16384;
static constexpr size_t kGtLevel2Requests = (size_t)1 << 20;
static constexpr int kNoMem = -1;       // internal: an allocation of the GT path failed
static constexpr int kOverBudget = -2;  // internal: a table level exceeds hg_set_table_budget
static int gt_forced_level() {
  static const int lvl = [] {
    const char* p = getenv("HG_AGG_PATH");
    if (p && strcmp(p, "g2") == 0) return 0;
    const char* e = getenv("HG_GT_LEVEL");
    if (!e) return -1;
    const int v = atoi(e);
    return v >= 0 && v <= 2 ? v : -1;
  }();
  return lvl;
}
// the registry's G2 membership count, waiting for its check if still running
static int resolve_subgroup(hg_ctx* c) {
  if (!c->sub_pending) return HG_OK;
  int cnt = 0;
  HG_CHECK(c, hipEventSynchronize(c->ev_sub));
  HG_CHECK(c, hipMemcpy(&cnt, c->sub_count.p, sizeof cnt, hipMemcpyDeviceToHost));
  c->reg_non_g2 = (size_t)cnt;
  c->sub_pending = false;
  return HG_OK;
}
// the highest table level the registry may use (the membership check must be resolved)
static int gt_max_level(const hg_ctx* c) {
  if (c->reg_non_g2 || c->sub_pending) return 0;
  const int top = c->nreg <= kGtMaxRegistry ? 2 : 1;
  return top < c->gt_cap ? top : c->gt_cap;
}

// an allocation of the GT path: out of device memory -> kNoMem (the caller
// falls back to a lower level), any other failure -> HG_ERR_DEVICE
#define HG_GT_ALLOC(ctx, expr)                                                     \
  do {                                                                             \
    hipError_t e_ = (expr);                                                        \
    if (e_ == hipErrorOutOfMemory) {                                               \
      (void)hipGetLastError(); /* not sticky: keep it out of check_launch */       \
      return kNoMem;                                                               \
    }                                                                              \
    if (e_ != hipSuccess) {                                                        \
      (ctx)->err = std::string(#expr) + ": " + hipGetErrorString(e_);              \
      return HG_ERR_DEVICE;                                                        \
    }                                                                              \
  } while (0)

// bytes of the tables of `level` (cumulative) for an n-key registry
static size_t gt_block_count(const hg_ctx* c, int* cnt) {
  size_t total = 0;
  for (int k = 4; k <= c->block_levels && k < 24; k++) {
    const size_t v = (c->nreg + ((size_t)1 << k) - 1) >> k;
    if (cnt) cnt[k] = (int)v;
    total += v;
  }
  return total;
}
static size_t gt_table_bytes(const hg_ctx* c, int level) {
  const size_t n = c->nreg, nwin8 = (n + 7) / 8, nwin16 = (n + 15) / 16;
  size_t b = 0;
  if (level >= 1) b += (n + nwin8 * 256 + gt_block_count(c, nullptr)) * sizeof(Gt);
  if (level >= 2) b += nwin16 * 65536 * sizeof(Gt);
  return b;
}

static size_t alt_table_bytes(const hg_ctx* c) {
  const TableSet& t = c->alt;
  return (t.gt_key.cap + t.gt_w8.cap + t.gt_win.cap + t.gt_blk.cap) * sizeof(Gt);
}
// frees the cached message's tables (its hash stays); false if it held none
static bool drop_alt_tables(hg_ctx* c) {
  if (alt_table_bytes(c) == 0) return false;
  release_tables(c->alt);
  return true;
}

// builds the tables up to `level` on stream s (inside a submission); kNoMem /
// kOverBudget before any launch of the level that could not be held. The
// budget covers both messages' tables.
static int build_gt_locked(hg_ctx* c, hipStream_t s, int level) {
  const int n = (int)c->nreg;
  const int nwin8 = (n + 7) / 8, nwin16 = (n + 15) / 16;
  if (c->gt_level < 1 && level >= 1) {
    if (gt_table_bytes(c, 1) + alt_table_bytes(c) > c->table_budget) return kOverBudget;
    int cnt[24] = {0};
    const size_t total = gt_block_count(c, cnt);
    int base = 0;
    for (int k = 4; k <= c->block_levels && k < 24; k++) {
      c->gt_bi.base[k] = base;
      base += cnt[k];
    }
    HG_GT_ALLOC(c, c->gt_key.ensure(n));
    HG_GT_ALLOC(c, c->gt_w8.ensure((size_t)nwin8 * 256));
    if (total) HG_GT_ALLOC(c, c->gt_blk.ensure(total));
    launch_gt_keys(c->reg.p, n, c->d_lines, c->d_h, c->gt_key.p, s);
    launch_gt_windows8(c->gt_key.p, n, c->gt_w8.p, nwin8, s);
    for (int k = 4; k <= c->block_levels && k < 24; k++) {
      if (k == 4) launch_gt_blocks(c->gt_w8.p + 255, 256, nwin8, c->gt_blk.p + c->gt_bi.base[4], cnt[4], s);
      else launch_gt_blocks(c->gt_blk.p + c->gt_bi.base[k - 1], 1, cnt[k - 1], c->gt_blk.p + c->gt_bi.base[k], cnt[k], s);
    }
    int rc = check_launch(c);
    if (rc) return rc;
    c->gt_level = 1;
  }
  if (c->gt_level < 2 && level >= 2) {
    if (gt_table_bytes(c, 2) + alt_table_bytes(c) > c->table_budget) return kOverBudget;
    HG_GT_ALLOC(c, c->gt_win.ensure((size_t)nwin16 * 65536));
    launch_gt_windows16(c->gt_w8.p, nwin8, c->gt_win.p, nwin16, s);
    int rc = check_launch(c);
    if (rc) return rc;
    c->gt_level = 2;
  }
  return HG_OK;
}

// caps the context's table level at `cap` and frees the tables above it; an
// out-of-memory cap also holds across later budget changes (oom_cap)
static void gt_lower_cap(hg_ctx* c, int cap, bool oom) {
  if (cap < 0) cap = 0;
  if (cap < c->gt_cap) c->gt_cap = cap;
  if (oom && cap < c->oom_cap) c->oom_cap = cap;
  if (c->gt_cap < 2) c->gt_win.release();
  if (c->gt_cap < 1) {
    c->gt_key.release();
    c->gt_w8.release();
    c->gt_blk.release();
  }
  if (c->gt_level > c->gt_cap) c->gt_level = c->gt_cap;
}

// builds up to `level` (lowering it to what fits: the cached message's tables
// go first, then the cap); HG_OK with `level` = what was built
static int build_fitting_locked(hg_ctx* c, hipStream_t s, int& level) {
  while (level > c->gt_level) {
    int rc = build_gt_locked(c, s, level);
    if (rc == kNoMem || rc == kOverBudget) {
      if (drop_alt_tables(c)) continue;
      gt_lower_cap(c, c->gt_level < level ? c->gt_level : level - 1, rc == kNoMem);
      level = level < c->gt_cap ? level : c->gt_cap;
      continue;
    }
    if (rc) return rc;
  }
  return HG_OK;
}

// the table level an aggregate submission of n requests runs at (counting
// them towards the volume policy)
static int gt_submission_level(hg_ctx* c, size_t n) {
  if (c->hash_eof || c->nreg == 0) return 0;
  // a GT level needs the registry's G2 membership (resolved only then)
  const bool wants_gt = c->pinned_level > 0 || c->gt_level > 0 || c->gt_requests + n >= kGtLevel1Requests;
  if (wants_gt && resolve_subgroup(c) != HG_OK) return 0;
  const int top = gt_max_level(c);
  if (c->pinned_level >= 0) return c->pinned_level < top ? c->pinned_level : top;
  c->gt_requests += n;
  int want = c->gt_requests >= kGtLevel2Requests ? 2 : (c->gt_requests >= kGtLevel1Requests ? 1 : 0);
  if (want < c->gt_level) want = c->gt_level;
  return want < top ? want : top;
}

// GT fold workspaces. A request of b bits has at most 8 nonzero 8-bit (4
// 16-bit) windows per registry-aligned 64-bit word of its range, plus the
// block term of a complemented fold.
// Fold schedule: terms per chunk and k_gt_chunks workgroups (HG_GT_CHUNK /
// HG_GT_GRID override them for tuning runs).
static int env_int(const char* name, int def, int lo, int hi) {
  const char* e = getenv(name);
  const int v = e ? atoi(e) : def;
  return v >= lo && v <= hi ? v : def;
}
static int gt_chunk() {
  static const int chunk = env_int("HG_GT_CHUNK", kGtChunk, 1, 64);
  return chunk;
}
static size_t fold_terms_bound(size_t bitlen) { return 8 * ((bitlen + 7 + 63) / 64) + 1; }
// capacity of a batch's term and chunk lists
struct FoldCaps {
  size_t terms = 0, chunks = 0;
  void add(size_t bitlen) {
    const size_t m = fold_terms_bound(bitlen);
    terms += m;
    chunks += (m + gt_chunk() - 1) / gt_chunk();
  }
};
// device-resident requests: their sizes are unknown on the host, every
// request is bounded by the registry
static FoldCaps fold_caps_worst(const hg_ctx* c, size_t n) {
  FoldCaps one;
  one.add(c->nreg);
  FoldCaps all;
  all.terms = one.terms * n;
  all.chunks = one.chunks * n;
  return all;
}
static int ensure_gt_fold(hg_ctx* c, Ws& ws, size_t n, const FoldCaps& caps, GtWork& w) {
  static const int grid = env_int("HG_GT_GRID", 4096, 64, 65536);
  if (caps.chunks > (size_t)INT32_MAX || caps.terms > (size_t)INT32_MAX) return kNoMem;
  HG_GT_ALLOC(c, ws.gt_plan.ensure(n));
  HG_GT_ALLOC(c, ws.gt_hdr.ensure(1));
  HG_GT_ALLOC(c, ws.gt_terms.ensure(caps.terms));
  HG_GT_ALLOC(c, ws.gt_ord.ensure(caps.chunks));
  HG_GT_ALLOC(c, ws.gt_multi.ensure(2 * n));
  HG_GT_ALLOC(c, ws.gt_partial.ensure(caps.chunks));
  HG_GT_ALLOC(c, ws.gt_y.ensure(n));
  w.plan = ws.gt_plan.p;
  w.hdr = ws.gt_hdr.p;
  w.terms = ws.gt_terms.p;
  w.ord = ws.gt_ord.p;
  w.cap = (int)caps.chunks;
  w.multi = ws.gt_multi.p;
  w.partial = ws.gt_partial.p;
  const size_t per_wg = kGtChunkTeams;
  // no more chunk workgroups than the batch can have chunks (a small batch
  // would otherwise launch thousands of workgroups that exit at once)
  const size_t need = (caps.chunks + per_wg - 1) / per_wg;
  w.chunk_grid = (int)(need < (size_t)grid ? (need ? need : 1) : (size_t)grid);
  w.chunk = gt_chunk();
  return HG_OK;
}

// The tables of `level` and the fold workspaces of one submission (inside it,
// on stream s). Lowers `level` for what the device cannot hold: tables that do
// not fit cap the context (tables never get smaller for this registry), fold
// workspaces that do not fit send this submission to the G2 fold only.
// may_build = false (service lanes): run at the built level at most; builds
// happen between batches, with the lanes drained (hg_lane_build_level)
static int gt_acquire(hg_ctx* c, Ws& ws, hipStream_t s, size_t n, const FoldCaps& caps, int& level, GtWork& w,
                      bool may_build = true) {
  if (!may_build && level > c->gt_level) level = c->gt_level;
  if (level > 0 && c->gt_level < level) {
    int rc = build_fitting_locked(c, s, level);
    if (rc) return rc;
  }
  if (level > 0) {
    int rc = ensure_gt_fold(c, ws, n, caps, w);
    if (rc == kNoMem) level = 0;
    else if (rc) return rc;
  }
  return HG_OK;
}

// The fold beside the pairing kernel (default; hg_set_fold_overlap(ctx, 0) or
// HG_GT_OVERLAP=0 for new contexts runs them one after the other, with the
// comparison inside k_verify_sig): k_verify_sig at one wave per SIMD leaves
// issue slots (and LDS for one fold workgroup per CU) for the fold's waves.
static bool gt_overlap() {
  static const bool on = env_int("HG_GT_OVERLAP", 1, 0, 1) != 0;
  return on;
}
static hipError_t ensure_side(Ws& ws) {
  hipError_t e = hipSuccess;
  if (!ws.side) e = hipStreamCreateWithFlags(&ws.side, hipStreamNonBlocking);
  if (e == hipSuccess && !ws.ev_fork) e = hipEventCreateWithFlags(&ws.ev_fork, hipEventDisableTiming);
  if (e == hipSuccess && !ws.ev_join) e = hipEventCreateWithFlags(&ws.ev_join, hipEventDisableTiming);
  return e;
}

// the level check of processing.go:350-352 on the device
__global__ void k_level_codes(const hg_request* r, int n, uint32_t nreg, int32_t* out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  bool ok = r[i].bitlen == r[i].level_size && (uint64_t)r[i].offset + r[i].bitlen <= nreg;
  out[i] = ok ? HG_OK : HG_ERR_LEVEL;
}

// The Combine fold and (verify) the pairing check of n requests, device
// pointers, on stream s; d_lvl holds the level codes and is updated in place
// (nullptr: computed here when the flow needs them). caps: the fold's list
// capacities (nullptr: bounded by the registry size).
// d_bits (nullable): the verdict bitset of the codes, written in the same
// submission (hg_pack_verdicts_device's layout)
// lane (nullable): a service lane's submission — its own workspaces, outside
// the context's submission chain, never building tables.
static int aggregate_device_locked(hg_ctx* c, const hg_request* d_reqs, size_t n, const uint64_t* d_words,
                                   const uint8_t* d_sigs, int32_t* d_codes, uint8_t* d_agg, int32_t* d_lvl,
                                   bool verify, hipStream_t s, const FoldCaps* caps = nullptr,
                                   uint8_t* d_bits = nullptr, hg_lane* lane = nullptr) {
  if (verify && !c->has_msg) {
    c->err = "hg_set_message was not called";
    return HG_ERR_ARG;
  }
  Ws& ws = lane ? lane->ws : c->ws;
  Submission sub(c, s);
  if (!lane) HG_CHECK(c, sub.start());
  // GT path: the verdict needs no aggregate key in G2; the G2 fold still runs
  // when the caller wants the aggregate keys' marshals
  int level = verify ? gt_submission_level(c, n) : 0;
  GtWork gw{};
  if (level > 0) {
    const FoldCaps fc = caps ? *caps : fold_caps_worst(c, n);
    int rc = gt_acquire(c, ws, s, n, fc, level, gw, lane == nullptr);
    if (rc) return rc;
  }
  const bool use_gt = level > 0;
  const bool g2_fold = !use_gt || d_agg;
  if (g2_fold) {
    HG_CHECK(c, ws.checks.ensure(n));
    HG_CHECK(c, ws.order.ensure(n));
    HG_CHECK(c, ws.agg_ws.ensure(n * agg_partial_bytes() + agg_fixed_bytes()));
  }
  if (d_agg) HG_CHECK(c, ws.pts2.ensure(n));
  if (!d_lvl) HG_CHECK(c, ws.codes_c.ensure(n));
  if (verify) {
    HG_CHECK(c, ws.pts1.ensure(n));
    HG_CHECK(c, ws.codes_b.ensure(n));
  }
  gw.win_bits = level == 2 ? 16 : 8;
  PhaseTimer all(c, HG_PHASE_SUBMIT, s);
  if (use_gt && !g2_fold) {
    // GT path, verdicts only: level check, signature decode and the fold's
    // counters in one launch, then the fold and the check on d_codes
    const bool overlap = lane ? lane->overlap : c->overlap;
    if (overlap) {
      HG_CHECK(c, ensure_side(ws));
      HG_CHECK(c, ws.gt_fe.ensure(n));
      if (sig12_for(lane ? lane->pad : true, n)) HG_CHECK(c, ws.sig_lines.ensure(sig12_lines_bytes((int)n)));
    }
    if (overlap) {
      // s:    pairing (decodes its signatures) ............ -> wait -> compare
      // side: wait -> prologue (codes, counters), plan, chunks, combine -> join
      HG_CHECK(c, hipEventRecord(ws.ev_fork, s));
      PhaseTimer t(c, HG_PHASE_VERIFY, s);
      if (sig12_for(lane ? lane->pad : true, n))
        launch_sig_pairing12(d_sigs, c->flavor, (int)n, c->d_lines, (Fp*)ws.sig_lines.p, ws.gt_fe.p, s,
                             lane ? lane->pad : true);
      else
        // the two-wave latency form for the context's own submissions (one
        // batch at a time); lanes keep batches in flight, where twice the
        // waves per check costs throughput (HG_SIG_W2_LANE_MAX: A/B)
        launch_sig_pairing(d_sigs, c->flavor, (int)n, c->d_lines, ws.gt_fe.p, s, lane ? lane->pad : true,
                           lane ? lane->w2_max : kSigW2MaxN);
      t.stop();
      HG_CHECK(c, hipStreamWaitEvent(ws.side, ws.ev_fork, 0));
      launch_agg_prologue(d_reqs, (int)n, (uint32_t)c->nreg, d_sigs, c->flavor, ws.pts1.p, d_codes, (int*)gw.hdr,
                          (int)(sizeof(GtHdr) / sizeof(int)), ws.side);
      PhaseTimer fold(c, HG_PHASE_AGGREGATE, ws.side);
      launch_gt_fold(d_reqs, (int)n, d_words, d_codes, (int)c->nreg, c->block_levels,
                     level == 2 ? c->gt_win.p : c->gt_w8.p, c->gt_blk.p, c->gt_bi, gw, ws.gt_y.p, false, ws.side);
      fold.stop();
      HG_CHECK(c, hipEventRecord(ws.ev_join, ws.side));
      HG_CHECK(c, hipStreamWaitEvent(s, ws.ev_join, 0));
      if (d_bits) launch_gt_compare_bits(ws.gt_fe.p, ws.gt_y.p, (int)n, d_codes, d_bits, s);
      else launch_gt_compare(ws.gt_fe.p, ws.gt_y.p, (int)n, d_codes, s);
      all.stop();
      int rc = check_launch(c);
      if (rc) return rc;
      if (!lane) HG_CHECK(c, sub.finish());
      return HG_OK;
    }
    launch_agg_prologue(d_reqs, (int)n, (uint32_t)c->nreg, d_sigs, c->flavor, ws.pts1.p, d_codes, (int*)gw.hdr,
                        (int)(sizeof(GtHdr) / sizeof(int)), s);
    PhaseTimer fold(c, HG_PHASE_AGGREGATE, s);
    launch_gt_fold(d_reqs, (int)n, d_words, d_codes, (int)c->nreg, c->block_levels,
                   level == 2 ? c->gt_win.p : c->gt_w8.p, c->gt_blk.p, c->gt_bi, gw, ws.gt_y.p, false, s);
    fold.stop();
    PhaseTimer t(c, HG_PHASE_VERIFY, s);
    launch_verify_sig(ws.pts1.p, (int)n, c->d_lines, ws.gt_y.p, d_codes, s);
    t.stop();
    if (d_bits) launch_pack_verdicts(d_codes, (int)n, d_bits, s);
    all.stop();
    int rc = check_launch(c);
    if (rc) return rc;
    if (!lane) HG_CHECK(c, sub.finish());
    return HG_OK;
  }
  if (!d_lvl) {
    d_lvl = ws.codes_c.p;
    k_level_codes<<<nb(n), 256, 0, s>>>(d_reqs, (int)n, (uint32_t)c->nreg, d_lvl);
  }
  PhaseTimer fold(c, HG_PHASE_AGGREGATE, s);
  if (g2_fold)
    launch_aggregate(c->wsum.p, (int)c->nreg, c->blocks.p, c->block_base.data(), c->block_levels, d_reqs, (int)n,
                     d_words, ws.order.p, ws.agg_ws.p, ws.checks.p, d_lvl, s);
  if (use_gt)
    launch_gt_fold(d_reqs, (int)n, d_words, d_lvl, (int)c->nreg, c->block_levels,
                   level == 2 ? c->gt_win.p : c->gt_w8.p, c->gt_blk.p, c->gt_bi, gw, ws.gt_y.p, true, s);
  fold.stop();
  if (d_agg) {
    launch_extract_pk(ws.checks.p, (int)n, ws.pts2.p, s);
    launch_encode_g2(ws.pts2.p, (int)n, d_agg, s);
  }
  if (verify) {
    launch_decode_g1(d_sigs, (int)n, c->flavor, ws.pts1.p, ws.codes_b.p, s);
    k_agg_codes<<<nb(n), 256, 0, s>>>(ws.codes_b.p, d_lvl, c->hash_eof ? 1 : 0, (int)n, d_codes);
    if (use_gt) {
      PhaseTimer t(c, HG_PHASE_VERIFY, s);
      launch_verify_sig(ws.pts1.p, (int)n, c->d_lines, ws.gt_y.p, d_codes, s);
      t.stop();
    } else if (!c->hash_eof) {
      launch_sig_into_checks(ws.pts1.p, (int)n, ws.checks.p, s);
      PhaseTimer t(c, HG_PHASE_VERIFY, s);
      launch_verify(ws.checks.p, (int)n, c->d_lines, c->d_h, d_codes, s);
      t.stop();
    }
  }
  if (d_bits) launch_pack_verdicts(d_codes, (int)n, d_bits, s);
  all.stop();
  int rc = check_launch(c);
  if (rc) return rc;
  if (!lane) HG_CHECK(c, sub.finish());
  return HG_OK;
}

static int aggregate_host_locked(hg_ctx* c, const hg_request* reqs, size_t n, const uint64_t* words, size_t nwords,
                                 const uint8_t* sigs, int32_t* codes, uint8_t* agg_out, bool verify) {
  HG_CHECK(c, hipSetDevice(c->device));
  std::vector<int32_t> lvl;
  level_codes(c, reqs, n, lvl);
  FoldCaps caps;  // exact bounds: the host knows every request's size
  for (size_t i = 0; i < n; i++) {
    if (lvl[i] != HG_OK) continue;
    if ((size_t)reqs[i].word_offset + (reqs[i].bitlen + 63) / 64 > nwords) {
      c->err = "request words out of range";
      return HG_ERR_ARG;
    }
    caps.add(reqs[i].bitlen);
  }
  HG_CHECK(c, c->reqs.ensure(n));
  HG_CHECK(c, c->words.ensure(nwords ? nwords : 1));
  HG_CHECK(c, c->codes_a.ensure(n));
  HG_CHECK(c, c->ws.codes_c.ensure(n));
  uint8_t* d_agg = nullptr;
  if (agg_out) {
    HG_CHECK(c, c->bytes_a.ensure(n * 128));
    d_agg = c->bytes_a.p;
  }
  if (verify) HG_CHECK(c, c->bytes_b.ensure(n * 64));
  Submission sub(c, c->stream);
  HG_CHECK(c, sub.start());
  HG_CHECK(c, hipMemcpyAsync(c->reqs.p, reqs, n * sizeof(hg_request), hipMemcpyHostToDevice, c->stream));
  if (nwords) HG_CHECK(c, hipMemcpyAsync(c->words.p, words, nwords * 8, hipMemcpyHostToDevice, c->stream));
  HG_CHECK(c, hipMemcpyAsync(c->ws.codes_c.p, lvl.data(), n * 4, hipMemcpyHostToDevice, c->stream));
  if (verify) HG_CHECK(c, hipMemcpyAsync(c->bytes_b.p, sigs, n * 64, hipMemcpyHostToDevice, c->stream));
  int rc = aggregate_device_locked(c, c->reqs.p, n, c->words.p, verify ? c->bytes_b.p : nullptr, c->codes_a.p, d_agg,
                                   c->ws.codes_c.p, verify, c->stream, &caps);
  if (rc) return rc;
  if (agg_out) HG_CHECK(c, hipMemcpyAsync(agg_out, d_agg, n * 128, hipMemcpyDeviceToHost, c->stream));
  HG_CHECK(c, hipMemcpyAsync(codes, verify ? c->codes_a.p : c->ws.codes_c.p, n * 4, hipMemcpyDeviceToHost, c->stream));
  HG_CHECK(c, sub.finish());
  HG_CHECK(c, hipStreamSynchronize(c->stream));
  if (agg_out) {
    // the reference has no aggregate for level errors / empty bitsets: zero them
    for (size_t i = 0; i < n; i++)
      if (lvl[i] != HG_OK || codes[i] == HG_ERR_EMPTY_AGG) memset(agg_out + 128 * i, 0, 128);
  }
  return HG_OK;
}

static int sign_locked(hg_ctx* c, const uint8_t* scalars_be, size_t n, uint8_t* sigs_out) {
  if (!c->has_msg) {
    c->err = "hg_set_message was not called";
    return HG_ERR_ARG;
  }
  if (c->hash_eof) return HG_ERR_HASH_EOF;
  if (n == 0) return HG_OK;
  HG_CHECK(c, hipSetDevice(c->device));
  HG_CHECK(c, c->bytes_a.ensure(n * 64));
  HG_CHECK(c, c->bytes_b.ensure(n * 32));
  HG_CHECK(c, c->ws.pts1.ensure(n));
  Submission sub(c, c->stream);
  HG_CHECK(c, sub.start());
  HG_CHECK(c, hipMemcpyAsync(c->bytes_b.p, scalars_be, n * 32, hipMemcpyHostToDevice, c->stream));
  launch_g1_mul(c->d_h, c->bytes_b.p, (int)n, c->ws.pts1.p, c->stream);
  launch_encode_g1(c->ws.pts1.p, (int)n, c->bytes_a.p, c->stream);
  int rc = check_launch(c);
  if (rc) return rc;
  HG_CHECK(c, hipMemcpyAsync(sigs_out, c->bytes_a.p, n * 64, hipMemcpyDeviceToHost, c->stream));
  HG_CHECK(c, sub.finish());
  HG_CHECK(c, hipStreamSynchronize(c->stream));
  return HG_OK;
}

extern "C" {

int hg_version(void) { return 2; }

const char* hg_code_string(int code, int flavor) { return code_text(code, flavor); }

const char* hg_processing_error_string(int code, int flavor) { return processing_text(code, flavor); }

int hg_context_simds(hg_ctx* c) {
  if (!c) return 0;
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device) != hipSuccess) return 0;
  return 4 * cus;  // CDNA: four SIMDs per compute unit
}

int hg_context_flavor(hg_ctx* c) { return c ? c->flavor : -1; }

const char* hg_last_error(hg_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int hg_create(int device, int flavor, hg_ctx** out) {
  if (!out || (flavor != HG_FLAVOR_GO && flavor != HG_FLAVOR_CF)) return HG_ERR_ARG;
  *out = nullptr;
  hg_ctx* c = new hg_ctx();
  c->device = device;
  c->flavor = flavor;
  c->pinned_level = gt_forced_level();
  c->overlap = gt_overlap();
  c->verify_split = env_int("HG_VERIFY_SPLIT", 0, 0, 1) != 0;
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipMalloc(&c->d_lines, sizeof(LineCoef) * kNumLines);
  if (e == hipSuccess) e = hipMalloc(&c->d_h, sizeof(PointG1));
  if (e == hipSuccess) e = hipMalloc(&c->d_k, sizeof(uint32_t) * 8);
  if (e != hipSuccess) {
    fprintf(stderr, "hg_create: %s\n", hipGetErrorString(e));
    release_all(c);
    delete c;
    return HG_ERR_DEVICE;
  }
  launch_g2_lines(c->d_lines, c->stream);
  if (check_launch(c) != HG_OK || hipStreamSynchronize(c->stream) != hipSuccess) {
    fprintf(stderr, "hg_create: %s\n", c->err.c_str());
    release_all(c);
    delete c;
    return HG_ERR_DEVICE;
  }
  *out = c;
  return HG_OK;
}

void hg_destroy(hg_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->ws.side) (void)hipStreamSynchronize(c->ws.side);
  if (c->last_ev) (void)hipEventSynchronize(c->last_ev);  // a submission on a caller stream
  release_all(c);
  delete c;
}

int hg_sync(hg_ctx* c) {
  if (!c) return HG_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  HG_CHECK(c, hipSetDevice(c->device));
  HG_CHECK(c, hipStreamSynchronize(c->stream));
  if (c->last_ev) HG_CHECK(c, hipEventSynchronize(c->last_ev));
  return HG_OK;
}

int hg_set_message(hg_ctx* c, const uint8_t* msg, size_t len) {
  if (!c || (!msg && len)) return HG_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  return set_message_locked(c, msg, len);
}

int hg_registry_load(hg_ctx* c, const uint8_t* pks, size_t n, int32_t* codes) {
  if (!c || (!pks && n)) return HG_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  HG_CHECK(c, hipSetDevice(c->device));
  // until every table is rebuilt the context has no registry: a failure below
  // leaves it empty (every aggregate request then fails its range check)
  c->nreg = 0;
  c->block_levels = 0;
  c->gt_level = 0;
  c->gt_requests = 0;
  c->alt.gt_level = 0;  // both messages' tables are e(H, .) of the old registry
  c->alt.gt_requests = 0;
  c->gt_cap = 2;
  c->oom_cap = 2;
  // the previous registry's membership check must be done before its buffer is reused
  if (c->sub_pending) HG_CHECK(c, hipEventSynchronize(c->ev_sub));
  c->sub_pending = false;
  c->reg_non_g2 = 0;
  Submission sub(c, c->stream);
  HG_CHECK(c, sub.start());
  HG_CHECK(c, hipStreamSynchronize(c->stream));
  HG_CHECK(c, c->reg.ensure(n));
  HG_CHECK(c, c->bytes_a.ensure(n * 128));
  HG_CHECK(c, c->codes_a.ensure(n));
  HG_CHECK(c, hipMemcpyAsync(c->bytes_a.p, pks, n * 128, hipMemcpyHostToDevice, c->stream));
  launch_decode_g2(c->bytes_a.p, (int)n, c->flavor, c->reg.p, c->codes_a.p, c->stream);
  int rc = check_launch(c);
  if (rc) return rc;
  std::vector<int32_t> h(n);
  if (n) HG_CHECK(c, hipMemcpyAsync(h.data(), c->codes_a.p, n * 4, hipMemcpyDeviceToHost, c->stream));
  HG_CHECK(c, hipStreamSynchronize(c->stream));
  int bad = 0;
  for (size_t i = 0; i < n; i++) bad |= h[i] != HG_OK;
  if (codes && n) memcpy(codes, h.data(), n * 4);
  if (bad) {
    c->err = "registry contains keys that fail to unmarshal";
    return HG_ERR_PK_UNMARSHAL;
  }
  // go flavor: x/crypto accepts any on-twist key (bn256/go/bn256.go:113-120);
  // count the keys outside G2 on the side stream (cf rejected them in the
  // decode above); the decode is complete (synchronised above)
  bool pending = false;
  if (c->flavor == HG_FLAVOR_GO && n) {
    HG_CHECK(c, ensure_side(c->ws));
    if (!c->ev_sub) HG_CHECK(c, hipEventCreateWithFlags(&c->ev_sub, hipEventDisableTiming));
    HG_CHECK(c, c->sub_count.ensure(1));
    HG_CHECK(c, hipMemsetAsync(c->sub_count.p, 0, sizeof(int), c->ws.side));
    launch_g2_subgroup(c->reg.p, (int)n, c->sub_count.p, c->ws.side);
    rc = check_launch(c);
    if (rc) return rc;
    HG_CHECK(c, hipEventRecord(c->ev_sub, c->ws.side));
    (void)hipStreamQuery(c->ws.side);  // flush: the check runs now, beside whatever follows
    pending = true;
  }
  // sums of the aligned power-of-two blocks (Handel's level ranges), level by level
  int K = 0;
  while (K < 23 && ((size_t)1 << K) < n) K++;
  std::vector<size_t> nbk(K + 1, 0);
  nbk[0] = n;
  size_t total = 0;
  for (int k = 1; k <= K; k++) {
    nbk[k] = (n + ((size_t)1 << k) - 1) >> k;
    c->block_base[k] = (int)total;
    total += nbk[k];
  }
  if (total) {
    HG_CHECK(c, c->blocks.ensure(total));
    for (int k = 1; k <= K; k++) {
      const PointG2* src = k == 1 ? c->reg.p : c->blocks.p + c->block_base[k - 1];
      launch_block_sums(src, (int)nbk[k - 1], c->blocks.p + c->block_base[k], (int)nbk[k], c->stream);
    }
    rc = check_launch(c);
    if (rc) return rc;
  }
  const size_t nwin = (n + 7) / 8;
  if (nwin) {
    HG_CHECK(c, c->wsum.ensure(nwin * 256));
    launch_window_sums(c->reg.p, (int)n, c->wsum.p, (int)nwin, c->stream);
    rc = check_launch(c);
    if (rc) return rc;
  }
  HG_CHECK(c, sub.finish());
  HG_CHECK(c, hipStreamSynchronize(c->stream));
  c->block_levels = K;
  c->nreg = n;
  c->sub_pending = pending;
  return HG_OK;
}

// builds the tables up to `want` (-1: the highest the registry, the pin and
// the device allow), synchronously
static int prepare_aggregate_locked(hg_ctx* c, int want = -1) {
  if (!c->has_msg || c->nreg == 0) {
    c->err = "hg_prepare_aggregate: needs a message and a registry";
    return HG_ERR_ARG;
  }
  if (c->hash_eof) return HG_ERR_HASH_EOF;
  int src = resolve_subgroup(c);
  if (src) return src;
  int level = gt_max_level(c);
  if (c->pinned_level >= 0 && c->pinned_level < level) level = c->pinned_level;
  if (want >= 0 && want < level) level = want;
  if (c->gt_level >= level) return HG_OK;
  HG_CHECK(c, hipSetDevice(c->device));
  Submission sub(c, c->stream);
  HG_CHECK(c, sub.start());
  // the highest level the device (and the table budget) can hold
  int rc = build_fitting_locked(c, c->stream, level);
  if (rc) return rc;
  HG_CHECK(c, sub.finish());
  HG_CHECK(c, hipStreamSynchronize(c->stream));
  return HG_OK;
}

int hg_prepare_aggregate(hg_ctx* c) {
  if (!c) return HG_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  return prepare_aggregate_locked(c);
}

int hg_prepare_aggregate_msg(hg_ctx* c, const uint8_t* msg, size_t len) {
  if (!c || (!msg && len)) return HG_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  int rc = set_message_locked(c, msg, len);
  if (rc) return rc;
  return prepare_aggregate_locked(c);
}

int hg_set_aggregate_level(hg_ctx* c, int level) {
  if (!c || level < -1 || level > 2) return HG_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  c->pinned_level = level;
  return HG_OK;
}

int hg_set_fold_overlap(hg_ctx* c, int on) {
  if (!c) return HG_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  c->overlap = on != 0;
  return HG_OK;
}

int hg_set_verify_split(hg_ctx* c, int on) {
  if (!c) return HG_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  c->verify_split = on != 0;
  return HG_OK;
}

int hg_set_table_budget(hg_ctx* c, size_t bytes) {
  if (!c) return HG_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  c->table_budget = bytes;
  // drop the built tables the new budget no longer covers (the cached
  // message's first); the cap is re-evaluated against the budget by the next
  // build, but never above what an out-of-memory failure left (oom_cap)
  if (gt_table_bytes(c, c->gt_level) + alt_table_bytes(c) > bytes) drop_alt_tables(c);
  if (c->gt_level >= 1 && gt_table_bytes(c, c->gt_level) > bytes)
    gt_lower_cap(c, gt_table_bytes(c, 1) <= bytes ? 1 : 0, false);
  c->gt_cap = c->oom_cap;
  return HG_OK;
}

size_t hg_registry_non_g2(hg_ctx* c) {
  if (!c) return 0;
  std::lock_guard<std::mutex> g(c->mu);
  if (resolve_subgroup(c) != HG_OK) return 0;
  return c->reg_non_g2;
}

int hg_aggregate_tables(hg_ctx* c) {
  if (!c) return 0;
  std::lock_guard<std::mutex> g(c->mu);
  return c->gt_level;
}

size_t hg_registry_size(hg_ctx* c) {
  if (!c) return 0;
  std::lock_guard<std::mutex> g(c->mu);
  return c->nreg;
}

int hg_verify_batch_device(hg_ctx* c, const uint8_t* d_pks, const uint8_t* d_sigs, size_t n, int32_t* d_codes,
                           void* stream) {
  if (!c || (n && (!d_pks || !d_sigs || !d_codes)) || n > (size_t)INT32_MAX) return HG_ERR_ARG;
  if (n == 0) return HG_OK;
  std::lock_guard<std::mutex> g(c->mu);
  HG_CHECK(c, hipSetDevice(c->device));
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  return verify_batch_device_locked(c, d_pks, d_sigs, n, d_codes, s);
}

int hg_pack_verdicts_device(hg_ctx* c, const int32_t* d_codes, size_t n, uint8_t* d_bits, void* stream) {
  if (!c || (n && (!d_codes || !d_bits)) || n > (size_t)INT32_MAX) return HG_ERR_ARG;
  if (n == 0) return HG_OK;
  std::lock_guard<std::mutex> g(c->mu);
  HG_CHECK(c, hipSetDevice(c->device));
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  Submission sub(c, s);
  HG_CHECK(c, sub.start());
  launch_pack_verdicts(d_codes, (int)n, d_bits, s);
  int rc = check_launch(c);
  if (rc) return rc;
  HG_CHECK(c, sub.finish());
  return HG_OK;
}

int hg_verify_batch(hg_ctx* c, const uint8_t* pks, const uint8_t* sigs, size_t n, int32_t* codes) {
  if (!c || (n && (!pks || !sigs || !codes)) || n > (size_t)INT32_MAX) return HG_ERR_ARG;
  if (n == 0) return HG_OK;
  std::lock_guard<std::mutex> g(c->mu);
  return verify_batch_host_locked(c, pks, sigs, n, codes);
}

int hg_verify_batch_msg(hg_ctx* c, const uint8_t* msg, size_t len, const uint8_t* pks, const uint8_t* sigs, size_t n,
                        int32_t* codes) {
  if (!c || (!msg && len) || (n && (!pks || !sigs || !codes)) || n > (size_t)INT32_MAX) return HG_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  int rc = set_message_locked(c, msg, len);
  if (rc != HG_OK && rc != HG_ERR_HASH_EOF) return rc;
  if (n == 0) return HG_OK;
  return verify_batch_host_locked(c, pks, sigs, n, codes);
}

int hg_verify_aggregate_device(hg_ctx* c, const hg_request* d_reqs, size_t n, const uint64_t* d_words,
                               const uint8_t* d_sigs, int32_t* d_codes, uint8_t* d_agg_pk_out, void* stream) {
  if (!c || (n && (!d_reqs || !d_sigs || !d_codes)) || n > (size_t)INT32_MAX) return HG_ERR_ARG;
  if (n == 0) return HG_OK;
  std::lock_guard<std::mutex> g(c->mu);
  HG_CHECK(c, hipSetDevice(c->device));
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  return aggregate_device_locked(c, d_reqs, n, d_words, d_sigs, d_codes, d_agg_pk_out, nullptr, true, s);
}

int hg_verify_aggregate_device_bits(hg_ctx* c, const hg_request* d_reqs, size_t n, const uint64_t* d_words,
                                    const uint8_t* d_sigs, int32_t* d_codes, uint8_t* d_bits, void* stream) {
  if (!c || (n && (!d_reqs || !d_sigs || !d_codes || !d_bits)) || n > (size_t)INT32_MAX) return HG_ERR_ARG;
  if (n == 0) return HG_OK;
  std::lock_guard<std::mutex> g(c->mu);
  HG_CHECK(c, hipSetDevice(c->device));
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  return aggregate_device_locked(c, d_reqs, n, d_words, d_sigs, d_codes, nullptr, nullptr, true, s, nullptr, d_bits);
}

int hg_verify_aggregate(hg_ctx* c, const hg_request* reqs, size_t n, const uint64_t* words, size_t nwords,
                        const uint8_t* sigs, int32_t* codes, uint8_t* agg_pk_out) {
  if (!c || (n && (!reqs || !sigs || !codes)) || n > (size_t)INT32_MAX) return HG_ERR_ARG;
  if (n == 0) return HG_OK;
  std::lock_guard<std::mutex> g(c->mu);
  return aggregate_host_locked(c, reqs, n, words, nwords, sigs, codes, agg_pk_out, true);
}

int hg_verify_aggregate_msg(hg_ctx* c, const uint8_t* msg, size_t len, const hg_request* reqs, size_t n,
                            const uint64_t* words, size_t nwords, const uint8_t* sigs, int32_t* codes,
                            uint8_t* agg_pk_out) {
  if (!c || (!msg && len) || (n && (!reqs || !sigs || !codes)) || n > (size_t)INT32_MAX) return HG_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  int rc = set_message_locked(c, msg, len);
  if (rc != HG_OK && rc != HG_ERR_HASH_EOF) return rc;
  if (n == 0) return HG_OK;
  return aggregate_host_locked(c, reqs, n, words, nwords, sigs, codes, agg_pk_out, true);
}

int hg_verify_multisig(hg_ctx* c, const uint32_t* bitlens, const uint32_t* word_offsets, size_t n,
                       const uint64_t* words, size_t nwords, const uint8_t* sigs, int32_t* codes) {
  if (!c || (n && (!bitlens || !word_offsets || !sigs || !codes)) || n > (size_t)INT32_MAX) return HG_ERR_ARG;
  if (n == 0) return HG_OK;
  std::lock_guard<std::mutex> g(c->mu);
  // crypto.go:121-124: the bitset must span the registry; the rest is
  // verifySignature over the range [0, N) (crypto.go:125-136)
  std::vector<hg_request> reqs(n);
  for (size_t i = 0; i < n; i++) reqs[i] = hg_request{0u, bitlens[i], (uint32_t)c->nreg, word_offsets[i]};
  int rc = aggregate_host_locked(c, reqs.data(), n, words, nwords, sigs, codes, nullptr, true);
  if (rc) return rc;
  for (size_t i = 0; i < n; i++)
    if (bitlens[i] != c->nreg) codes[i] = HG_ERR_MULTI_SIZES;
  return HG_OK;
}

int hg_aggregate_pk(hg_ctx* c, const hg_request* reqs, size_t n, const uint64_t* words, size_t nwords,
                    uint8_t* agg_pk_out, int32_t* codes) {
  if (!c || (n && (!reqs || !agg_pk_out || !codes)) || n > (size_t)INT32_MAX) return HG_ERR_ARG;
  if (n == 0) return HG_OK;
  std::lock_guard<std::mutex> g(c->mu);
  return aggregate_host_locked(c, reqs, n, words, nwords, nullptr, codes, agg_pk_out, false);
}

int hg_combine_g1(hg_ctx* c, const uint8_t* a, const uint8_t* b, size_t n, uint8_t* out, int32_t* codes) {
  if (!c || (n && (!a || !b || !out || !codes)) || n > (size_t)INT32_MAX) return HG_ERR_ARG;
  if (n == 0) return HG_OK;
  std::lock_guard<std::mutex> g(c->mu);
  HG_CHECK(c, hipSetDevice(c->device));
  HG_CHECK(c, c->bytes_a.ensure(n * 64));
  HG_CHECK(c, c->bytes_b.ensure(n * 64));
  HG_CHECK(c, c->ws.pts1.ensure(n));
  HG_CHECK(c, c->pts1b.ensure(n));
  HG_CHECK(c, c->codes_a.ensure(n));
  HG_CHECK(c, c->ws.codes_b.ensure(n));
  HG_CHECK(c, c->ws.codes_c.ensure(n));
  Submission sub(c, c->stream);
  HG_CHECK(c, sub.start());
  HG_CHECK(c, hipMemcpyAsync(c->bytes_a.p, a, n * 64, hipMemcpyHostToDevice, c->stream));
  HG_CHECK(c, hipMemcpyAsync(c->bytes_b.p, b, n * 64, hipMemcpyHostToDevice, c->stream));
  launch_decode_g1(c->bytes_a.p, (int)n, c->flavor, c->ws.pts1.p, c->codes_a.p, c->stream);
  launch_decode_g1(c->bytes_b.p, (int)n, c->flavor, c->pts1b.p, c->ws.codes_b.p, c->stream);
  launch_merge_codes(c->codes_a.p, c->ws.codes_b.p, (int)n, c->ws.codes_c.p, c->stream);
  launch_g1_combine(c->ws.pts1.p, c->pts1b.p, (int)n, c->bytes_a.p, c->stream);
  int rc = check_launch(c);
  if (rc) return rc;
  HG_CHECK(c, hipMemcpyAsync(out, c->bytes_a.p, n * 64, hipMemcpyDeviceToHost, c->stream));
  HG_CHECK(c, hipMemcpyAsync(codes, c->ws.codes_c.p, n * 4, hipMemcpyDeviceToHost, c->stream));
  HG_CHECK(c, sub.finish());
  HG_CHECK(c, hipStreamSynchronize(c->stream));
  return HG_OK;
}

int hg_combine_g2(hg_ctx* c, const uint8_t* a, const uint8_t* b, size_t n, uint8_t* out, int32_t* codes) {
  if (!c || (n && (!a || !b || !out || !codes)) || n > (size_t)INT32_MAX) return HG_ERR_ARG;
  if (n == 0) return HG_OK;
  std::lock_guard<std::mutex> g(c->mu);
  HG_CHECK(c, hipSetDevice(c->device));
  HG_CHECK(c, c->bytes_a.ensure(n * 128 * 2));
  HG_CHECK(c, c->ws.pts2.ensure(n * 3));
  HG_CHECK(c, c->codes_a.ensure(n));
  HG_CHECK(c, c->ws.codes_b.ensure(n));
  HG_CHECK(c, c->ws.codes_c.ensure(n));
  uint8_t* d = c->bytes_a.p;
  Submission sub(c, c->stream);
  HG_CHECK(c, sub.start());
  HG_CHECK(c, hipMemcpyAsync(d, a, n * 128, hipMemcpyHostToDevice, c->stream));
  HG_CHECK(c, hipMemcpyAsync(d + n * 128, b, n * 128, hipMemcpyHostToDevice, c->stream));
  launch_decode_g2(d, (int)n, c->flavor, c->ws.pts2.p, c->codes_a.p, c->stream);
  launch_decode_g2(d + n * 128, (int)n, c->flavor, c->ws.pts2.p + n, c->ws.codes_b.p, c->stream);
  launch_merge_codes(c->codes_a.p, c->ws.codes_b.p, (int)n, c->ws.codes_c.p, c->stream);
  launch_g2_combine(c->ws.pts2.p, c->ws.pts2.p + n, (int)n, c->ws.pts2.p + 2 * n, c->stream);
  launch_encode_g2(c->ws.pts2.p + 2 * n, (int)n, d, c->stream);
  int rc = check_launch(c);
  if (rc) return rc;
  HG_CHECK(c, hipMemcpyAsync(out, d, n * 128, hipMemcpyDeviceToHost, c->stream));
  HG_CHECK(c, hipMemcpyAsync(codes, c->ws.codes_c.p, n * 4, hipMemcpyDeviceToHost, c->stream));
  HG_CHECK(c, sub.finish());
  HG_CHECK(c, hipStreamSynchronize(c->stream));
  return HG_OK;
}

int hg_pair(hg_ctx* c, const uint8_t* g1s, const uint8_t* g2s, size_t n, uint8_t* gt_out, int32_t* codes) {
  if (!c || (n && (!g1s || !g2s || !gt_out || !codes)) || n > (size_t)INT32_MAX) return HG_ERR_ARG;
  if (n == 0) return HG_OK;
  std::lock_guard<std::mutex> g(c->mu);
  HG_CHECK(c, hipSetDevice(c->device));
  HG_CHECK(c, c->bytes_a.ensure(n * 384));
  HG_CHECK(c, c->bytes_b.ensure(n * 64));
  HG_CHECK(c, c->ws.pts1.ensure(n));
  HG_CHECK(c, c->ws.pts2.ensure(n));
  HG_CHECK(c, c->codes_a.ensure(n));
  HG_CHECK(c, c->ws.codes_b.ensure(n));
  HG_CHECK(c, c->ws.codes_c.ensure(n));
  Submission sub(c, c->stream);
  HG_CHECK(c, sub.start());
  HG_CHECK(c, hipMemcpyAsync(c->bytes_a.p, g2s, n * 128, hipMemcpyHostToDevice, c->stream));
  HG_CHECK(c, hipMemcpyAsync(c->bytes_b.p, g1s, n * 64, hipMemcpyHostToDevice, c->stream));
  launch_decode_g2(c->bytes_a.p, (int)n, HG_FLAVOR_GO, c->ws.pts2.p, c->codes_a.p, c->stream);
  launch_decode_g1(c->bytes_b.p, (int)n, HG_FLAVOR_GO, c->ws.pts1.p, c->ws.codes_b.p, c->stream);
  launch_merge_codes(c->codes_a.p, c->ws.codes_b.p, (int)n, c->ws.codes_c.p, c->stream);
  launch_pair(c->ws.pts1.p, c->ws.pts2.p, (int)n, c->d_lines, c->bytes_a.p, c->stream);
  int rc = check_launch(c);
  if (rc) return rc;
  HG_CHECK(c, hipMemcpyAsync(gt_out, c->bytes_a.p, n * 384, hipMemcpyDeviceToHost, c->stream));
  HG_CHECK(c, hipMemcpyAsync(codes, c->ws.codes_c.p, n * 4, hipMemcpyDeviceToHost, c->stream));
  HG_CHECK(c, sub.finish());
  HG_CHECK(c, hipStreamSynchronize(c->stream));
  return HG_OK;
}

int hg_keygen(hg_ctx* c, const uint8_t* scalars_be, size_t n, uint8_t* pks_out) {
  if (!c || (n && (!scalars_be || !pks_out)) || n > (size_t)INT32_MAX) return HG_ERR_ARG;
  if (n == 0) return HG_OK;
  std::lock_guard<std::mutex> g(c->mu);
  HG_CHECK(c, hipSetDevice(c->device));
  HG_CHECK(c, c->bytes_a.ensure(n * 128));
  HG_CHECK(c, c->bytes_b.ensure(n * 32));
  HG_CHECK(c, c->ws.pts2.ensure(n));
  Submission sub(c, c->stream);
  HG_CHECK(c, sub.start());
  HG_CHECK(c, hipMemcpyAsync(c->bytes_b.p, scalars_be, n * 32, hipMemcpyHostToDevice, c->stream));
  launch_g2_mul_base(c->bytes_b.p, (int)n, c->ws.pts2.p, c->stream);
  launch_encode_g2(c->ws.pts2.p, (int)n, c->bytes_a.p, c->stream);
  int rc = check_launch(c);
  if (rc) return rc;
  HG_CHECK(c, hipMemcpyAsync(pks_out, c->bytes_a.p, n * 128, hipMemcpyDeviceToHost, c->stream));
  HG_CHECK(c, sub.finish());
  HG_CHECK(c, hipStreamSynchronize(c->stream));
  return HG_OK;
}

int hg_sign(hg_ctx* c, const uint8_t* scalars_be, size_t n, uint8_t* sigs_out) {
  if (!c || (n && (!scalars_be || !sigs_out)) || n > (size_t)INT32_MAX) return HG_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  return sign_locked(c, scalars_be, n, sigs_out);
}

int hg_sign_msg(hg_ctx* c, const uint8_t* msg, size_t len, const uint8_t* scalars_be, size_t n, uint8_t* sigs_out) {
  if (!c || (!msg && len) || (n && (!scalars_be || !sigs_out)) || n > (size_t)INT32_MAX) return HG_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  int rc = set_message_locked(c, msg, len);
  if (rc != HG_OK) return rc;
  return sign_locked(c, scalars_be, n, sigs_out);
}

int hg_debug_fp12(hg_ctx* c, int op, const uint8_t* a, const uint8_t* b, size_t n, uint8_t* out) {
  if (!c || (n && (!a || !b || !out)) || n > (size_t)INT32_MAX) return HG_ERR_ARG;
  if (n == 0) return HG_OK;
  std::lock_guard<std::mutex> g(c->mu);
  HG_CHECK(c, hipSetDevice(c->device));
  HG_CHECK(c, c->bytes_a.ensure(n * 384 * 3));
  uint8_t* d = c->bytes_a.p;
  Submission sub(c, c->stream);
  HG_CHECK(c, sub.start());
  HG_CHECK(c, hipMemcpyAsync(d, a, n * 384, hipMemcpyHostToDevice, c->stream));
  HG_CHECK(c, hipMemcpyAsync(d + n * 384, b, n * 384, hipMemcpyHostToDevice, c->stream));
  launch_fp12_op(op, d, d + n * 384, (int)n, d + 2 * n * 384, c->stream);
  int rc = check_launch(c);
  if (rc) return rc;
  HG_CHECK(c, hipMemcpyAsync(out, d + 2 * n * 384, n * 384, hipMemcpyDeviceToHost, c->stream));
  HG_CHECK(c, sub.finish());
  HG_CHECK(c, hipStreamSynchronize(c->stream));
  return HG_OK;
}

int hg_sig_pairing_device(hg_ctx* c, const uint8_t* d_sigs, size_t n, uint8_t* d_fe, int kernel, void* stream) {
  if (!c || (n && (!d_sigs || !d_fe)) || n > (size_t)INT32_MAX || kernel < 0 || kernel > 4) return HG_ERR_ARG;
  if ((kernel == 2 || kernel == 3) && n > (size_t)kSig12MaxN) return HG_ERR_ARG;  // k_sig_lines: 4 n threads in int
  if (n == 0) return HG_OK;
  std::lock_guard<std::mutex> g(c->mu);
  HG_CHECK(c, hipSetDevice(c->device));
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  Submission sub(c, s);
  HG_CHECK(c, sub.start());
  const bool pad = (kernel & 1) == 0;
  if (kernel == 4) {
    launch_sig_pairing_w2(d_sigs, c->flavor, (int)n, c->d_lines, (Gt*)d_fe, s);
  } else if (kernel >= 2) {
    HG_CHECK(c, c->ws.sig_lines.ensure(sig12_lines_bytes((int)n)));
    launch_sig_pairing12(d_sigs, c->flavor, (int)n, c->d_lines, (Fp*)c->ws.sig_lines.p, (Gt*)d_fe, s, pad);
  } else {
    launch_sig_pairing(d_sigs, c->flavor, (int)n, c->d_lines, (Gt*)d_fe, s, pad, 0);
  }
  int rc = check_launch(c);
  if (rc) return rc;
  HG_CHECK(c, sub.finish());
  return HG_OK;
}

int hg_diag_read(hg_ctx* c, uint64_t* out, size_t n) {
  if (!c || !out) return HG_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  HG_CHECK(c, hipSetDevice(c->device));
  HG_CHECK(c, hipStreamSynchronize(c->stream));
  if (c->last_ev) HG_CHECK(c, hipEventSynchronize(c->last_ev));
  return diag_read(out, n) == 0 ? HG_OK : HG_ERR_ARG;
}

// ---------------------------------------------------------------- packet intake
static bool packet_args_ok(const hg_ctx* c, size_t n, size_t stride) {
  // slot word offsets (2n slots of `stride` words) are 32-bit
  return n <= (size_t)INT32_MAX / 2 && stride >= pkt_stride_words(c->nreg) && stride <= (size_t)INT32_MAX &&
         (n == 0 || 2 * n <= (size_t)UINT32_MAX / stride);
}

size_t hg_packet_stride_words(hg_ctx* c) {
  if (!c) return 0;
  std::lock_guard<std::mutex> g(c->mu);
  return pkt_stride_words(c->nreg);
}

int hg_parse_packets_device(hg_ctx* c, const uint8_t* d_pool, size_t pool_len, const hg_packet* d_pkts, size_t n,
                            size_t stride_words, hg_request* d_reqs, uint64_t* d_words, uint8_t* d_sigs,
                            int32_t* d_codes, void* stream) {
  if (!c || (n && (!d_pkts || !d_reqs || !d_words || !d_sigs || !d_codes)) || (pool_len && !d_pool)) return HG_ERR_ARG;
  if (n == 0) return HG_OK;
  std::lock_guard<std::mutex> g(c->mu);
  if (!packet_args_ok(c, n, stride_words)) return HG_ERR_ARG;
  HG_CHECK(c, hipSetDevice(c->device));
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  Submission sub(c, s);
  HG_CHECK(c, sub.start());
  launch_parse_packets(d_pool, pool_len, d_pkts, (int)n, (uint32_t)c->nreg, c->flavor, (int)stride_words, d_reqs,
                       d_words, d_sigs, d_codes, s);
  int rc = check_launch(c);
  if (rc) return rc;
  HG_CHECK(c, sub.finish());
  return HG_OK;
}

int hg_parse_packets(hg_ctx* c, const uint8_t* pool, size_t pool_len, const hg_packet* pkts, size_t n,
                     size_t stride_words, hg_request* reqs, uint64_t* words, uint8_t* sigs, int32_t* codes) {
  if (!c || (n && (!pkts || !reqs || !words || !sigs || !codes)) || (pool_len && !pool)) return HG_ERR_ARG;
  if (n == 0) return HG_OK;
  for (size_t i = 0; i < n; i++) {
    const hg_packet& p = pkts[i];
    if ((uint64_t)p.ms_off + p.ms_len > pool_len ||
        ((p.flags & HG_PKT_HAS_IND) && (uint64_t)p.ind_off + p.ind_len > pool_len))
      return HG_ERR_ARG;
  }
  std::lock_guard<std::mutex> g(c->mu);
  if (!packet_args_ok(c, n, stride_words)) return HG_ERR_ARG;
  HG_CHECK(c, hipSetDevice(c->device));
  const size_t nw = 2 * n * stride_words;
  HG_CHECK(c, c->bytes_a.ensure(pool_len ? pool_len : 1));
  HG_CHECK(c, c->bytes_b.ensure(2 * n * 64));
  HG_CHECK(c, c->pkts.ensure(n));
  HG_CHECK(c, c->reqs.ensure(2 * n));
  HG_CHECK(c, c->words.ensure(nw));
  HG_CHECK(c, c->codes_a.ensure(2 * n));
  Submission sub(c, c->stream);
  HG_CHECK(c, sub.start());
  if (pool_len) HG_CHECK(c, hipMemcpyAsync(c->bytes_a.p, pool, pool_len, hipMemcpyHostToDevice, c->stream));
  HG_CHECK(c, hipMemcpyAsync(c->pkts.p, pkts, n * sizeof(hg_packet), hipMemcpyHostToDevice, c->stream));
  launch_parse_packets(c->bytes_a.p, pool_len, c->pkts.p, (int)n, (uint32_t)c->nreg, c->flavor, (int)stride_words,
                       c->reqs.p, c->words.p, c->bytes_b.p, c->codes_a.p, c->stream);
  int rc = check_launch(c);
  if (rc) return rc;
  HG_CHECK(c, hipMemcpyAsync(reqs, c->reqs.p, 2 * n * sizeof(hg_request), hipMemcpyDeviceToHost, c->stream));
  HG_CHECK(c, hipMemcpyAsync(words, c->words.p, nw * sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream));
  HG_CHECK(c, hipMemcpyAsync(sigs, c->bytes_b.p, 2 * n * 64, hipMemcpyDeviceToHost, c->stream));
  HG_CHECK(c, hipMemcpyAsync(codes, c->codes_a.p, 2 * n * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
  HG_CHECK(c, sub.finish());
  HG_CHECK(c, hipStreamSynchronize(c->stream));
  return HG_OK;
}

int hg_packet_error(hg_ctx* c, int code, const hg_packet* p, char* buf, size_t cap) {
  if (!c || !p || (cap && !buf)) return -1;
  size_t nreg;
  int flavor;
  {
    std::lock_guard<std::mutex> g(c->mu);
    nreg = c->nreg;
    flavor = c->flavor;
  }
  if (code == HG_ERR_PKT_LEVEL) return snprintf(buf, cap, "invalid packet's level %d", (int)p->level);
  if (code == HG_ERR_PKT_ID_RANGE) {
    // partitioner.go:113-115 (the receiver's range at the packet's level)
    uint32_t lo = 0, hi = 0;
    (void)pkt_range_level(p->receiver, (uint32_t)nreg, (int)p->level, lo, hi);
    return snprintf(buf, cap, "globalID outside level's range. id=%d, min=%u, max=%u, level=%d", (int)p->origin, lo,
                    hi, (int)p->level);
  }
  return snprintf(buf, cap, "%s", hg_code_string(code, flavor));
}

size_t hg_context_bytes(hg_ctx* c) {
  if (!c) return 0;
  std::lock_guard<std::mutex> g(c->mu);
  size_t b = sizeof(LineCoef) * kNumLines + 2 * sizeof(PointG1) + 32;
  b += c->reg.cap * sizeof(PointG2) + c->blocks.cap * sizeof(PointG2) + c->wsum.cap * sizeof(PointG2);
  b += c->bytes_a.cap + c->bytes_b.cap + c->pts1b.cap * sizeof(PointG1);
  b += c->codes_a.cap * sizeof(int32_t) + c->reqs.cap * sizeof(hg_request) + c->words.cap * sizeof(uint64_t);
  b += (c->gt_key.cap + c->gt_w8.cap + c->gt_win.cap + c->gt_blk.cap) * sizeof(Gt) + alt_table_bytes(c);
  b += c->ws.bytes();
  for (const hg_lane* l : c->lanes) b += l->ws.bytes() + l->d_in.cap + l->d_codes.cap * sizeof(int32_t);
  b += c->sub_count.cap * sizeof(int) + c->pkts.cap * sizeof(hg_packet);
  return b;
}

int hg_timing_enable(hg_ctx* c, int on) {
  if (!c) return HG_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  c->timing = on != 0;
  return HG_OK;
}

int hg_timing_read_phase(hg_ctx* c, int phase, double* total_ms, int* launches) {
  if (!c || !total_ms || !launches || phase < 0 || phase >= HG_NUM_PHASES) return HG_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  HG_CHECK(c, hipSetDevice(c->device));
  double tot = 0;
  int k = 0;
  auto& ev = c->events[phase];
  int rc = HG_OK;
  for (auto& pr : ev) {
    float ms = 0;
    hipError_t e = hipEventSynchronize(pr.second);
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, pr.first, pr.second);
    if (e != hipSuccess && rc == HG_OK) {
      c->err = std::string("hg_timing_read_phase: ") + hipGetErrorString(e);
      rc = HG_ERR_DEVICE;
    }
    tot += ms;
    k++;
    (void)hipEventDestroy(pr.first);
    (void)hipEventDestroy(pr.second);
  }
  ev.clear();
  *total_ms = tot;
  *launches = k;
  return rc;
}

int hg_timing_read(hg_ctx* c, double* total_ms, int* launches) {
  return hg_timing_read_phase(c, HG_PHASE_VERIFY, total_ms, launches);
}

int hg_debug_fp_mul(hg_ctx* c, const uint32_t* a, const uint32_t* b, size_t n, uint32_t* out) {
  if (!c || (n && (!a || !b || !out)) || n > (size_t)INT32_MAX) return HG_ERR_ARG;
  if (n == 0) return HG_OK;
  std::lock_guard<std::mutex> g(c->mu);
  HG_CHECK(c, hipSetDevice(c->device));
  HG_CHECK(c, c->bytes_a.ensure(n * 32 * 3));
  uint32_t* da = (uint32_t*)c->bytes_a.p;
  Submission sub(c, c->stream);
  HG_CHECK(c, sub.start());
  HG_CHECK(c, hipMemcpyAsync(da, a, n * 32, hipMemcpyHostToDevice, c->stream));
  HG_CHECK(c, hipMemcpyAsync(da + 8 * n, b, n * 32, hipMemcpyHostToDevice, c->stream));
  launch_fp_mul(da, da + 8 * n, (int)n, da + 16 * n, c->stream);
  int rc = check_launch(c);
  if (rc) return rc;
  HG_CHECK(c, hipMemcpyAsync(out, da + 16 * n, n * 32, hipMemcpyDeviceToHost, c->stream));
  HG_CHECK(c, sub.finish());
  HG_CHECK(c, hipStreamSynchronize(c->stream));
  return HG_OK;
}

int hg_prepare_aggregate_level(hg_ctx* c, int level) {
  if (!c || level < 0 || level > 2) return HG_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  return prepare_aggregate_locked(c, level);
}

// ---------------------------------------------------------------- lanes
int hg_lane_create(hg_ctx* c, size_t max_batch, size_t max_words, int overlap, hg_lane** out) {
  if (!c || !out || max_batch == 0 || max_batch > (size_t)INT32_MAX || max_words > ((size_t)1 << 40))
    return HG_ERR_ARG;
  *out = nullptr;
  std::lock_guard<std::mutex> g(c->mu);
  HG_CHECK(c, hipSetDevice(c->device));
  hg_lane* l = new hg_lane();
  l->c = c;
  l->overlap = overlap != 0;
  l->max_batch = max_batch;
  l->max_words = max_words;
  // staging: requests | signatures | words, each 256-byte aligned
  const size_t bytes = ((max_batch * sizeof(hg_request) + 255) & ~(size_t)255) +
                       ((max_batch * 64 + 255) & ~(size_t)255) + max_words * 8 + 256;
  hipError_t e = hipStreamCreateWithFlags(&l->s, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&l->done, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&l->ev_in, hipEventDisableTiming);
  if (e == hipSuccess) e = hipHostMalloc(&l->h_in, bytes, hipHostMallocDefault);
  if (e == hipSuccess) e = hipHostMalloc(&l->h_codes, max_batch * sizeof(int32_t), hipHostMallocDefault);
  if (e == hipSuccess) e = l->d_in.ensure(bytes);
  if (e == hipSuccess) e = l->d_codes.ensure(max_batch);
  // every workspace at its largest now (max_batch requests over max_words
  // bitset words): a buffer that grew later would be freed and reallocated
  // between batches, and hipFree waits for the whole device
  const size_t n = max_batch;
  const size_t terms = 8 * (max_words + n) + n;  // sum of fold_terms_bound over the batch
  const size_t chunks = terms / (size_t)gt_chunk() + n;
  Ws& w = l->ws;
  if (e == hipSuccess) e = w.pts1.ensure(n);
  if (e == hipSuccess) e = w.codes_b.ensure(n);
  if (e == hipSuccess) e = w.codes_c.ensure(n);
  if (e == hipSuccess) e = w.checks.ensure(n);
  if (e == hipSuccess) e = w.order.ensure(n);
  if (e == hipSuccess) e = w.agg_ws.ensure(n * agg_partial_bytes() + agg_fixed_bytes());
  if (e == hipSuccess) e = w.gt_plan.ensure(n);
  if (e == hipSuccess) e = w.gt_hdr.ensure(1);
  if (e == hipSuccess) e = w.gt_terms.ensure(terms);
  if (e == hipSuccess) e = w.gt_ord.ensure(chunks);
  if (e == hipSuccess) e = w.gt_multi.ensure(2 * n);
  if (e == hipSuccess) e = w.gt_partial.ensure(chunks);
  if (e == hipSuccess) e = w.gt_y.ensure(n);
  if (e == hipSuccess) e = w.gt_fe.ensure(n);
  if (e == hipSuccess && sig12_for(true, n)) e = w.sig_lines.ensure(sig12_lines_bytes((int)n));
  if (e == hipSuccess && l->overlap) e = ensure_side(w);
  if (e != hipSuccess) {
    c->err = std::string("hg_lane_create: ") + hipGetErrorString(e);
    l->ws.release();
    l->d_in.release();
    l->d_codes.release();
    if (l->h_in) (void)hipHostFree(l->h_in);
    if (l->h_codes) (void)hipHostFree(l->h_codes);
    if (l->done) (void)hipEventDestroy(l->done);
    if (l->ev_in) (void)hipEventDestroy(l->ev_in);
    if (l->s) (void)hipStreamDestroy(l->s);
    delete l;
    return HG_ERR_DEVICE;
  }
  c->lanes.push_back(l);
  *out = l;
  return HG_OK;
}

void hg_lane_destroy(hg_lane* l) {
  if (!l) return;
  hg_ctx* c = l->c;
  std::lock_guard<std::mutex> g(c->mu);
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(l->s);
  if (l->ws.side) (void)hipStreamSynchronize(l->ws.side);
  for (size_t i = 0; i < c->lanes.size(); i++)
    if (c->lanes[i] == l) {
      c->lanes.erase(c->lanes.begin() + (long)i);
      break;
    }
  l->ws.release();
  l->d_in.release();
  l->d_codes.release();
  (void)hipHostFree(l->h_in);
  (void)hipHostFree(l->h_codes);
  (void)hipEventDestroy(l->done);
  (void)hipEventDestroy(l->ev_in);
  (void)hipStreamDestroy(l->s);
  delete l;
}

int hg_lane_stage(hg_lane* l, size_t n, size_t nwords, hg_request** reqs, uint8_t** sigs, uint64_t** words) {
  if (!l || !reqs || !sigs || !words || n == 0 || n > l->max_batch || nwords > l->max_words) return HG_ERR_ARG;
  l->n = n;
  l->nwords = nwords;
  l->off_sigs = (n * sizeof(hg_request) + 255) & ~(size_t)255;
  l->off_words = (l->off_sigs + n * 64 + 255) & ~(size_t)255;
  l->in_bytes = l->off_words + nwords * 8;
  *reqs = reinterpret_cast<hg_request*>(l->h_in);
  *sigs = l->h_in + l->off_sigs;
  *words = reinterpret_cast<uint64_t*>(l->h_in + l->off_words);
  return HG_OK;
}

int hg_lane_submit(hg_lane* l) {
  if (!l || l->n == 0) return HG_ERR_ARG;
  hg_ctx* c = l->c;
  const size_t n = l->n;
  const hg_request* h_reqs = reinterpret_cast<const hg_request*>(l->h_in);
  // exact fold capacities from the requests (what aggregate_host_locked does),
  // and no bitset read outside the staged words
  FoldCaps caps;
  for (size_t i = 0; i < n; i++) {
    const hg_request& r = h_reqs[i];
    if ((size_t)r.word_offset + ((size_t)r.bitlen + 63) / 64 > l->nwords) return HG_ERR_ARG;
    caps.add(r.bitlen);
  }
  std::lock_guard<std::mutex> g(c->mu);
  HG_CHECK(c, hipSetDevice(c->device));
  // after the context's last submission (a registry load, a hash, a table
  // build); the lanes' own batches are independent of each other
  if (c->last_ev) HG_CHECK(c, hipStreamWaitEvent(l->s, c->last_ev, 0));
  uint8_t* d = l->d_in.p;
  HG_CHECK(c, hipMemcpyAsync(d, l->h_in, l->in_bytes, hipMemcpyHostToDevice, l->s));
  int rc = aggregate_device_locked(c, reinterpret_cast<const hg_request*>(d), n,
                                   reinterpret_cast<const uint64_t*>(d + l->off_words), d + l->off_sigs,
                                   l->d_codes.p, nullptr, nullptr, true, l->s, &caps, nullptr, l);
  if (rc) return rc;
  HG_CHECK(c, hipMemcpyAsync(l->h_codes, l->d_codes.p, n * sizeof(int32_t), hipMemcpyDeviceToHost, l->s));
  HG_CHECK(c, hipEventRecord(l->done, l->s));
  l->recorded = true;
  (void)hipStreamQuery(l->s);  // flush: start now
  return HG_OK;
}

void* hg_lane_stream(hg_lane* l) { return l ? (void*)l->s : nullptr; }

int hg_lane_set_pairing_padding(hg_lane* l, int pad) {
  if (!l) return HG_ERR_ARG;
  hg_ctx* c = l->c;
  std::lock_guard<std::mutex> g(c->mu);
  // the unpadded lane runs the 12-lane kernel: its evaluated-line workspace
  // at the lane's largest batch now (never grown between batches)
  if (sig12_for(pad != 0, l->max_batch)) {
    HG_CHECK(c, hipSetDevice(c->device));
    HG_CHECK(c, hipStreamSynchronize(l->s));
    if (l->ws.side) HG_CHECK(c, hipStreamSynchronize(l->ws.side));
    HG_CHECK(c, l->ws.sig_lines.ensure(sig12_lines_bytes((int)l->max_batch)));
  }
  l->pad = pad != 0;
  return HG_OK;
}

int hg_lane_set_latency_form(hg_lane* l, int max_checks) {
  if (!l || max_checks < 0) return HG_ERR_ARG;
  std::lock_guard<std::mutex> g(l->c->mu);
  l->w2_max = max_checks < kSigW2MaxN ? max_checks : kSigW2MaxN;
  return HG_OK;
}

int hg_lane_submit_device(hg_lane* l, const hg_request* d_reqs, size_t n, const uint64_t* d_words,
                          const uint8_t* d_sigs, int32_t* d_codes, uint8_t* d_bits, void* stream) {
  if (!l || !d_reqs || !d_sigs || !d_codes || n == 0 || n > l->max_batch) return HG_ERR_ARG;
  hg_ctx* c = l->c;
  std::lock_guard<std::mutex> g(c->mu);
  HG_CHECK(c, hipSetDevice(c->device));
  hipStream_t caller = stream ? (hipStream_t)stream : c->stream;
  // after the caller's earlier work on `stream` (its inputs, its last reads of
  // d_codes / d_bits) and the context's last submission
  HG_CHECK(c, hipEventRecord(l->ev_in, caller));
  HG_CHECK(c, hipStreamWaitEvent(l->s, l->ev_in, 0));
  if (c->last_ev) HG_CHECK(c, hipStreamWaitEvent(l->s, c->last_ev, 0));
  const FoldCaps caps = fold_caps_worst(c, n);  // the device words are not visible to the host
  int rc = aggregate_device_locked(c, d_reqs, n, d_words, d_sigs, d_codes, nullptr, nullptr, true, l->s, &caps,
                                   d_bits, l);
  if (rc) return rc;
  HG_CHECK(c, hipEventRecord(l->done, l->s));
  l->recorded = true;
  HG_CHECK(c, hipStreamWaitEvent(caller, l->done, 0));  // the verdicts, in the caller's stream order
  return HG_OK;
}

int hg_lane_query(hg_lane* l) {
  if (!l) return -HG_ERR_ARG;
  if (!l->recorded) return 1;
  hipError_t e = hipEventQuery(l->done);
  if (e == hipSuccess) return 1;
  if (e == hipErrorNotReady) return 0;
  return -HG_ERR_DEVICE;
}

int hg_lane_wait(hg_lane* l) {
  if (!l) return HG_ERR_ARG;
  if (!l->recorded) return HG_OK;
  return hipEventSynchronize(l->done) == hipSuccess ? HG_OK : HG_ERR_DEVICE;
}

const int32_t* hg_lane_codes(hg_lane* l) { return l ? l->h_codes : nullptr; }

}  // extern "C"
