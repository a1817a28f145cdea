// hg_service.cpp — the GPU-owning verifier service (C ABI hg_service_* in
// include/handel_gpu.h; shared-memory layout in hg_shm.h; clients in
// hg_client.cpp).
//
// simul's single-host run puts P OS processes of k Handel instances each on
// one machine (simul/node/main.go:63-131); every instance's evaluator checks
// one multisignature at a time (processing.go:228-287 -> verifySignature
// :342-368). Giving each process its own GPU context means P copies of the
// registry and the GT tables, P batchers each seeing 1/P of the load, and
// one batch in flight per process. Here one dispatcher thread serves them
// all: it takes queued requests from the shared region, merges them into
// batches (one message per batch), keeps up to `lanes` batches in flight on
// the GPU at once (hg_lane_*: each lane its own stream and workspaces over
// the one set of tables), and returns every code to its client's channel.
//
// Dispatch rule: a batch goes out when a lane is free and either max_batch
// requests are queued or the oldest queued request has waited max_wait_us.
// The dispatcher spins while batches are in flight (completion latency is
// the point) and sleeps on the doorbell futex when idle.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <string>
#include <thread>
#include <vector>

#include "../../include/handel_gpu.h"
#include "hg_shm.h"

using namespace hgshm;
using Clock = std::chrono::steady_clock;

namespace {

// What executes a staged batch: the GPU (lanes of one context) or a CPU
// stand-in for protocol tests.
struct Exec {
  virtual ~Exec() = default;
  virtual int lanes() const = 0;
  virtual int stage(int lane, size_t n, size_t nwords, hg_request** r, uint8_t** s, uint64_t** w) = 0;
  virtual int submit(int lane) = 0;
  virtual int query(int lane) = 0;  // 1 done, 0 running, < 0 failed
  virtual const int32_t* codes(int lane) = 0;
  // the message of the next batches (every lane idle); prepare: build the
  // top table level now; returns HG_OK / HG_ERR_HASH_EOF or an error
  virtual int use_message(const uint8_t* m, size_t len, bool prepare) = 0;
  virtual int build_level(int level) = 0;  // every lane idle
  // pairing waves the device holds at one per SIMD, and the lane's latency
  // form for its next batch (hg_lane_set_latency_form)
  virtual int simds() const { return 1024; }
  virtual void latency_form(int, int) {}
};

struct GpuExec : Exec {
  hg_ctx* ctx;
  std::vector<hg_lane*> ln;
  bool warmed = false;
  explicit GpuExec(hg_ctx* c) : ctx(c) {}
  // one tiny batch per lane, waited for: every kernel of the path is loaded
  // and every lane's stream has run once before the first client's batch
  // (all lanes at once: one pairing kernel's time); needs the context's
  // message, else it waits for the first one
  void warm_up() {
    bool ok = true;
    for (hg_lane* l : ln) {
      hg_request* r = nullptr;
      uint8_t* s = nullptr;
      uint64_t* w = nullptr;
      ok = ok && hg_lane_stage(l, 1, 1, &r, &s, &w) == HG_OK;
      if (!ok) break;
      r[0] = hg_request{0, 1, 1, 0};
      w[0] = 1;
      memset(s, 0, 64);
      ok = hg_lane_submit(l) == HG_OK;
    }
    for (hg_lane* l : ln) (void)hg_lane_wait(l);
    warmed = ok;
  }
  ~GpuExec() override {
    for (hg_lane* l : ln) hg_lane_destroy(l);
  }
  int lanes() const override { return (int)ln.size(); }
  int stage(int i, size_t n, size_t nw, hg_request** r, uint8_t** s, uint64_t** w) override {
    return hg_lane_stage(ln[i], n, nw, r, s, w);
  }
  int submit(int i) override { return hg_lane_submit(ln[i]); }
  int query(int i) override { return hg_lane_query(ln[i]); }
  const int32_t* codes(int i) override { return hg_lane_codes(ln[i]); }
  int use_message(const uint8_t* m, size_t len, bool prepare) override {
    const int rc = prepare ? hg_prepare_aggregate_msg(ctx, m, len) : hg_set_message(ctx, m, len);
    if (rc == HG_OK && !warmed) warm_up();
    return rc;
  }
  int build_level(int level) override { return hg_prepare_aggregate_level(ctx, level); }
  int simd_count = 0;
  int simds() const override { return simd_count; }
  void latency_form(int i, int max_checks) override { (void)hg_lane_set_latency_form(ln[i], max_checks); }
};

// CPU stand-in (hg_service_create_echo): codes from the request bytes
struct EchoExec : Exec {
  struct Lane {
    std::vector<hg_request> reqs;
    std::vector<uint8_t> sigs;
    std::vector<uint64_t> words;
    std::vector<int32_t> codes;
    size_t n = 0;
    Clock::time_point due;
  };
  std::vector<Lane> ln;
  uint32_t nreg;
  std::chrono::microseconds delay;
  EchoExec(int lanes, size_t max_batch, size_t max_words, uint32_t nreg_, uint32_t delay_us)
      : ln(lanes), nreg(nreg_), delay(delay_us) {
    for (Lane& l : ln) {
      l.reqs.resize(max_batch);
      l.sigs.resize(64 * max_batch);
      l.words.resize(max_words ? max_words : 1);
      l.codes.resize(max_batch);
    }
  }
  int lanes() const override { return (int)ln.size(); }
  int stage(int i, size_t n, size_t nw, hg_request** r, uint8_t** s, uint64_t** w) override {
    Lane& l = ln[i];
    if (n > l.reqs.size() || nw > l.words.size()) return HG_ERR_ARG;
    l.n = n;
    *r = l.reqs.data();
    *s = l.sigs.data();
    *w = l.words.data();
    return HG_OK;
  }
  int submit(int i) override {
    Lane& l = ln[i];
    for (size_t k = 0; k < l.n; k++) {
      const hg_request& q = l.reqs[k];
      const uint8_t* sig = &l.sigs[64 * k];
      if (q.bitlen != q.level_size || (uint64_t)q.offset + q.bitlen > nreg) {
        l.codes[k] = HG_ERR_LEVEL;
        continue;
      }
      uint64_t x = 0, want = 0;
      for (uint32_t j = 0; j < (q.bitlen + 63) / 64; j++) x ^= l.words[q.word_offset + j];
      for (int b = 0; b < 8; b++) want |= (uint64_t)sig[1 + b] << (8 * b);
      l.codes[k] = x != want ? 77 : (sig[0] == 1 ? HG_ERR_SIG_INVALID : HG_OK);
    }
    l.due = Clock::now() + delay;
    return HG_OK;
  }
  int query(int i) override { return Clock::now() >= ln[i].due ? 1 : 0; }
  const int32_t* codes(int i) override { return ln[i].codes.data(); }
  int use_message(const uint8_t*, size_t, bool) override { return HG_OK; }
  int build_level(int) override { return HG_OK; }
};

// A queued request as intake() found it: every field the dispatcher uses is
// copied out of the shared slot once, when the slot turns Taken, so a client
// that rewrites its slot afterwards cannot change what is validated, sized or
// copied (processing.go:342-352: a bitset that does not fit its level is an
// error, never a crash). Only the bitset words and the signature are read from
// the slot later, once, at launch, sized by this copy.
struct Pending {
  uint32_t slot, gen, chan, msg, msg_gen;
  uint32_t offset, bitlen, level_size;
  Clock::time_point seen;
};

}  // namespace

struct hg_service {
  hg_service_config cfg{};
  std::string name;
  int fd = -1;
  View v;
  Exec* ex = nullptr;
  std::thread th;
  std::atomic<bool> stop{false};
  // dispatcher-local
  std::vector<uint32_t> tails;  // per channel: completions pushed
  std::vector<uint8_t> touched;
  std::deque<Pending> pending;
  struct LaneState {
    bool busy = false;
    std::vector<Pending> slots;
    int waves = 0;  // pairing waves of the batch in flight
  };
  std::vector<LaneState> lanes;
  int busy = 0;
  int cur_msg = -1;
  uint32_t cur_gen = 0;
  uint64_t msg_requests = 0;
  int built_level = 0;
  uint64_t max_in_flight = 0;
  Clock::time_point last_arrival;
  // requests released by finished batches whose clients have not submitted
  // again (cfg.follow): a closed-loop cohort is back when this reaches zero.
  // Counted per channel, so that only a resubmission from a channel whose
  // requests were released counts (open-loop arrivals from other channels do
  // not make the cohort look complete)
  uint64_t returning = 0;
  std::vector<uint32_t> released;  // per channel
  bool released_any = false;
  std::vector<Pending> take;
  // channels whose handle closed with requests in flight (kChanOrphaned):
  // adopted[ch] once the dispatcher has swept the ring the handle left
  std::vector<uint8_t> adopted;
  uint32_t seen_orphans = 0;
  // Service-side records (the shared words are client-writable, so nothing
  // the orphan path frees or releases rests on them alone):
  //  outstanding[ch]  requests of channel ch taken at intake, not yet finished
  //  owed_chan[id]    the channel whose ring the dispatcher pushed slot id
  //                   into (kNone once the slot is taken again), with the
  //                   slot generation it had at intake (owed_gen[id])
  static constexpr uint32_t kNone = 0xFFFFFFFFu;
  std::vector<uint32_t> outstanding;
  std::vector<uint32_t> owed_chan, owed_gen;
  // the two-wave latency form for the service's batches: off by default
  // (HG_SERVICE_W2=1 turns it on). Measured on the config-4 proxy it bought
  // no throughput and doubled p99 (profiles/r05sy_service_policy_ab.json:
  // 2.3-2.8 ms on vs 1.2-1.4 ms off, more and smaller batches)
  bool w2_policy = false;
#ifdef HG_SERVICE_TESTING
  uint32_t test_finish_us = 0;  // HG_SERVICE_TEST_FINISH_US
#endif
  static constexpr int kW2MaxChecks = 2048;  // the latency form's largest batch (bn256_gt.h kSigW2MaxN)

  bool intake();
  void complete(int lane, const int32_t* codes, int32_t fail);
  void finish_slots(const Pending* items, size_t n, const int32_t* codes, int32_t fail);
  void free_slot(uint32_t id, uint32_t ch);
  void maybe_release(uint32_t ch);
  void adopt(uint32_t ch);
  void sweep_orphans();
  void drain();
  void launch(int lane);
  void run();
};

// queued slots -> pending (in slot order within a bitmap word)
bool hg_service::intake() {
  bool any = false;
  const uint32_t words = v.h->nslots / 64;
  std::atomic<uint64_t>* q = v.queued_bits();
  const auto now = Clock::now();
  for (uint32_t w = 0; w < words; w++) {
    if (!q[w].load(std::memory_order_relaxed)) continue;
    uint64_t x = q[w].exchange(0, std::memory_order_acq_rel);
    while (x) {
      const uint32_t id = w * 64 + (uint32_t)__builtin_ctzll(x);
      x &= x - 1;
      Slot* s = v.slot(id);
      if (s->state.load(std::memory_order_acquire) != kSlotQueued) continue;
      s->state.store(kSlotTaken, std::memory_order_relaxed);
      Pending p{id, s->gen, s->chan, s->msg, s->msg_gen, s->offset, s->bitlen, s->level_size, now};
      pending.push_back(p);
      owed_chan[id] = kNone;
      if (p.chan < outstanding.size()) outstanding[p.chan]++;
      if (p.chan < released.size() && released[p.chan]) {
        released[p.chan]--;
        if (returning) returning--;
      }
      any = true;
    }
  }
  if (any) last_arrival = now;
  return any;
}

// a finished slot of an orphaned channel: nobody will collect it, so the
// dispatcher frees it; the channel is released once it owns no slot
void hg_service::free_slot(uint32_t id, uint32_t ch) {
  Slot* s = v.slot(id);
  owed_chan[id] = kNone;
  s->state.store(kSlotFree, std::memory_order_release);
  v.free_bits()[id / 64].fetch_or(1ull << (id % 64), std::memory_order_release);
  // the client-side count (what a live handle would have decremented),
  // never below zero whatever a client wrote there
  std::atomic<uint32_t>& in = v.chan(ch)->inflight;
  uint32_t x = in.load(std::memory_order_acquire);
  while (x && !in.compare_exchange_weak(x, x - 1, std::memory_order_acq_rel)) {
  }
  maybe_release(ch);
}

// an adopted channel is reusable once the service holds none of its requests
// (its own count) and no slot of it is claimed but not yet queued (the
// client-side count: a handle closed mid-submit); a new handle starts reading
// its ring at the tail published at that point, so it never sees a foreign
// completion
void hg_service::maybe_release(uint32_t ch) {
  if (!adopted[ch] || outstanding[ch] || v.chan(ch)->inflight.load(std::memory_order_acquire)) return;
#ifdef HG_SERVICE_TESTING
  // the invariant the race harness checks: nothing pushed to this ring is
  // left unpublished when the channel goes back to the pool
  if (touched[ch]) {
    fprintf(stderr, "hg_service: channel %u released with unpublished completions\n", ch);
    abort();
  }
#endif
  adopted[ch] = 0;
  v.chan(ch)->used.store(kChanFree, std::memory_order_release);
}

// takes over an orphaned channel: the completions pushed after its handle's
// last drain (ring positions [head, tail)) are freed here. The pending tail
// of a batch being finished is published first, so that the positions this
// walk frees are never published afterwards (a handle opened on
// the released channel would read them). head and the ring are client-written:
// a walk longer than the ring is a forged header and frees nothing, and a
// ring entry is freed only if the dispatcher itself pushed that slot, with
// that generation, into this channel's ring and it is still Done.
void hg_service::adopt(uint32_t ch) {
  Channel* c = v.chan(ch);
  if (touched[ch]) {
    touched[ch] = 0;
    c->tail.store(tails[ch], std::memory_order_seq_cst);
  }
  adopted[ch] = 1;
  const uint32_t cap = v.h->nslots;
  const uint32_t* ring = v.ring(ch);
  const uint32_t head = c->head, dist = tails[ch] - head;
  if (dist <= cap)
    for (uint32_t k = 0; k < dist; k++) {
      const uint32_t id = ring[(head + k) % cap];
      if (id >= cap || owed_chan[id] != ch) continue;
      Slot* s = v.slot(id);
      if (s->state.load(std::memory_order_acquire) == kSlotDone && s->gen == owed_gen[id]) free_slot(id, ch);
    }
  maybe_release(ch);
}

void hg_service::sweep_orphans() {
  const uint32_t o = v.h->orphans.load(std::memory_order_acquire);
  if (o == seen_orphans) return;
  seen_orphans = o;
  for (uint32_t ch = 0; ch < v.h->nchan; ch++)
    if (!adopted[ch] && v.chan(ch)->used.load(std::memory_order_acquire) == kChanOrphaned) adopt(ch);
}

// codes into the slots, slot ids into their channels' rings, one wake per
// channel (the channel is the one intake() recorded, not the slot's word now)
void hg_service::finish_slots(const Pending* items, size_t n, const int32_t* codes, int32_t fail) {
  if (n == 0) return;
  const uint32_t cap = v.h->nslots;
  for (size_t i = 0; i < n; i++) {
#ifdef HG_SERVICE_TESTING
    // the CPU race harness widens the windows between one completion and the
    // next and before the tails' publication (service_asan.cpp "race")
    if (test_finish_us && i) std::this_thread::sleep_for(std::chrono::microseconds(test_finish_us));
#endif
    const uint32_t id = items[i].slot, ch = items[i].chan;
    Slot* s = v.slot(id);
    s->code = codes ? codes[i] : fail;
    s->state.store(kSlotDone, std::memory_order_release);
    if (ch >= v.h->nchan) continue;
    if (outstanding[ch]) outstanding[ch]--;
    Channel* c = v.chan(ch);
    if (c->used.load(std::memory_order_acquire) == kChanOrphaned) {
      if (!adopted[ch]) adopt(ch);
      if (adopted[ch]) {
        free_slot(id, ch);
        continue;
      }
    }
    owed_chan[id] = ch;
    owed_gen[id] = items[i].gen;
    v.ring(ch)[tails[ch] % cap] = id;
    tails[ch]++;
    touched[ch] = 1;
  }
#ifdef HG_SERVICE_TESTING
  if (test_finish_us) std::this_thread::sleep_for(std::chrono::microseconds(test_finish_us));
#endif
  for (uint32_t ch = 0; ch < v.h->nchan; ch++) {
    if (!touched[ch]) continue;
    touched[ch] = 0;
    Channel* c = v.chan(ch);
    c->tail.store(tails[ch], std::memory_order_seq_cst);
    if (c->waiters.load(std::memory_order_seq_cst)) futex_wake(&c->tail);
  }
}

void hg_service::complete(int lane, const int32_t* codes, int32_t fail) {
  LaneState& L = lanes[lane];
  // the counters first: a client that sees its verdict (the tail's release
  // store in finish_slots) sees them counted
  v.h->batches.fetch_add(1, std::memory_order_relaxed);
  v.h->requests.fetch_add(L.slots.size(), std::memory_order_relaxed);
  finish_slots(L.slots.data(), L.slots.size(), codes, fail);
  for (const Pending& p : L.slots)
    if (p.chan < released.size()) released[p.chan]++;
  returning += L.slots.size();
  released_any = true;
  L.slots.clear();
  L.busy = false;
  busy--;
}

// waits for every batch in flight (message switches and table builds)
void hg_service::drain() {
  while (busy > 0) {
    for (int i = 0; i < (int)lanes.size(); i++) {
      if (!lanes[i].busy) continue;
      const int q = ex->query(i);
      if (q == 1) complete(i, ex->codes(i), 0);
      else if (q < 0) complete(i, nullptr, HG_ERR_DEVICE);
    }
    cpu_relax();
  }
}

void hg_service::launch(int lane) {
  const Pending first = pending.front();
  // the batch's message: pinned by its clients, so the entry is stable
  const Msg& m = v.h->msgs[first.msg < kMaxMsgs ? first.msg : 0];
  const bool msg_ok = first.msg < kMaxMsgs && m.gen == first.msg_gen &&
                      m.state.load(std::memory_order_acquire) == kMsgReady && m.len <= kMsgCap;
  if (!msg_ok) {  // a stale message reference: fail that request alone
    pending.pop_front();
    const int32_t code = HG_ERR_ARG;
    finish_slots(&first, 1, &code, 0);
    return;
  }
  if ((int)first.msg != cur_msg || first.msg_gen != cur_gen) {
    drain();
    const int rc = ex->use_message(m.bytes, m.len, cfg.prepare != 0);
    cur_msg = (int)first.msg;
    cur_gen = first.msg_gen;
    msg_requests = 0;
    built_level = cfg.prepare ? 2 : 0;
    if (rc != HG_OK && rc != HG_ERR_HASH_EOF) {
      fprintf(stderr, "hg_service: message setup failed (%d)\n", rc);
      cur_msg = -1;
      std::vector<Pending> ids;
      for (auto it = pending.begin(); it != pending.end();) {
        if (it->msg == first.msg && it->msg_gen == first.msg_gen) {
          ids.push_back(*it);
          it = pending.erase(it);
        } else {
          ++it;
        }
      }
      finish_slots(ids.data(), ids.size(), nullptr, HG_ERR_DEVICE);
      return;
    }
  }
  // up to max_batch requests of this message, in arrival order
  take.clear();
  size_t nwords = 0;
  const uint32_t max_bits = v.h->slot_words * 64;
  std::vector<Pending> bad;
  for (auto it = pending.begin(); it != pending.end() && take.size() < cfg.max_batch;) {
    if (it->msg != first.msg || it->msg_gen != first.msg_gen) {
      ++it;
      continue;
    }
    if (it->bitlen > max_bits) bad.push_back(*it);
    else {
      take.push_back(*it);
      nwords += (it->bitlen + 63) / 64;
    }
    it = pending.erase(it);
  }
  if (!bad.empty()) {
    std::vector<int32_t> codes(bad.size(), HG_ERR_ARG);
    finish_slots(bad.data(), bad.size(), codes.data(), 0);
  }
  if (take.empty()) return;
  // the volume policy (prepare = 0): the context's break-even thresholds
  msg_requests += take.size();
  if (!cfg.prepare) {
    const int want = msg_requests >= ((uint64_t)1 << 20) ? 2 : (msg_requests >= 16384 ? 1 : 0);
    if (want > built_level) {
      drain();
      (void)ex->build_level(want);  // what does not fit stays at the level below
      built_level = want;
    }
  }
  hg_request* r = nullptr;
  uint8_t* sg = nullptr;
  uint64_t* w = nullptr;
  int rc = ex->stage(lane, take.size(), nwords, &r, &sg, &w);
  if (rc == HG_OK) {
    uint32_t wo = 0;
    for (size_t i = 0; i < take.size(); i++) {
      const Pending& p = take[i];
      Slot* s = v.slot(p.slot);
      const uint32_t nw = (p.bitlen + 63) / 64;  // <= slot_words: checked above on the same copy
      r[i] = hg_request{p.offset, p.bitlen, p.level_size, wo};
      memcpy(sg + 64 * i, s->sig, 64);
      memcpy(w + wo, s->words(), 8ull * nw);
      wo += nw;
    }
    // with HG_SERVICE_W2=1: the two-wave latency form while the batches in
    // flight leave a SIMD for each of its waves (padded kernels: one wave per
    // SIMD), else the one-wave kernel (the default: always)
    const int n = (int)take.size(), one = (n + 3) / 4;
    int used = 0;
    for (const LaneState& o : lanes)
      if (o.busy) used += o.waves;
    const bool w2 = w2_policy && n <= kW2MaxChecks && used + 2 * one <= ex->simds();
    ex->latency_form(lane, w2 ? kW2MaxChecks : 0);
    lanes[lane].waves = w2 ? 2 * one : one;
    rc = ex->submit(lane);
  }
  LaneState& L = lanes[lane];
  L.slots.assign(take.begin(), take.end());
  L.busy = true;
  busy++;
  if ((uint64_t)busy > max_in_flight) max_in_flight = (uint64_t)busy;
  if (rc != HG_OK) complete(lane, nullptr, rc == HG_ERR_ARG ? HG_ERR_ARG : HG_ERR_DEVICE);
}

void hg_service::run() {
  const auto linger = std::chrono::microseconds(cfg.max_wait_us);
  const auto quiet = std::chrono::microseconds(cfg.quiet_us);
  Header* h = v.h;
  for (;;) {
    bool progress = false;
    for (int i = 0; i < (int)lanes.size(); i++) {
      if (!lanes[i].busy) continue;
      const int q = ex->query(i);
      if (q == 1) complete(i, ex->codes(i), 0);
      else if (q < 0) complete(i, nullptr, HG_ERR_DEVICE);
      else continue;
      progress = true;
    }
    progress |= intake();
    sweep_orphans();
    const bool stopping = stop.load(std::memory_order_acquire);
    while (!pending.empty()) {
      int free_lane = -1;
      for (int i = 0; i < (int)lanes.size() && free_lane < 0; i++)
        if (!lanes[i].busy) free_lane = i;
      if (free_lane < 0) break;
      const bool full = pending.size() >= cfg.max_batch;
      const auto now = Clock::now();
      const bool old = now - pending.front().seen >= linger;
      // a burst of resubmissions (the clients of a finished batch) has ended
      const bool calm = cfg.quiet_us && now - last_arrival >= quiet;
      // every request the finished batches released has been submitted again
      const bool back = cfg.follow && released_any && returning == 0;
      if (!full && !old && !calm && !back && !stopping) break;
      launch(free_lane);
      progress = true;
    }
    if (stopping && pending.empty() && busy == 0 && !intake()) break;
    if (progress) continue;
    if (busy > 0 || !pending.empty()) {
      cpu_relax();
      continue;
    }
    // idle: sleep until a client rings (the flag first, then one last look)
    const uint32_t bell = h->doorbell.load(std::memory_order_seq_cst);
    h->sleeping.store(1, std::memory_order_seq_cst);
    bool queued = false;
    std::atomic<uint64_t>* qb = v.queued_bits();
    for (uint32_t w = 0; w < h->nslots / 64 && !queued; w++) queued = qb[w].load(std::memory_order_seq_cst) != 0;
    queued = queued || h->orphans.load(std::memory_order_seq_cst) != seen_orphans;
    if (!queued && !stop.load(std::memory_order_acquire)) futex_wait(&h->doorbell, bell, 20000);
    h->sleeping.store(0, std::memory_order_seq_cst);
  }
}

namespace {

int create_common(const char* name, const hg_service_config* in, uint32_t nreg, uint32_t flavor,
                  hg_service** out, hg_service*& s) {
  if (!name || !out || name[0] != '/' || strlen(name) > 200) return HG_ERR_ARG;
  *out = nullptr;
  hg_service_config cfg;
  hg_service_config_init(&cfg);
  if (in) cfg = *in;
  if (cfg.slots == 0) cfg.slots = 8192;
  if (cfg.slot_bits == 0) cfg.slot_bits = nreg ? nreg : 64;
  if (cfg.channels == 0) cfg.channels = 256;
  if (cfg.lanes == 0) cfg.lanes = 8;
  if (cfg.max_batch == 0) cfg.max_batch = 4096;
  if (cfg.slots % 64 || cfg.slots > (1u << 22) || cfg.channels > 4096 || cfg.lanes > 64 ||
      cfg.slot_bits > (1u << 24) || cfg.max_batch > (1u << 20))
    return HG_ERR_ARG;
  const uint32_t slot_words = (cfg.slot_bits + 63) / 64;
  const Layout L = layout(cfg.slots, slot_words, cfg.channels);
  const int fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
  if (fd < 0) return HG_ERR_ARG;
  if (ftruncate(fd, (off_t)L.bytes) != 0) {
    close(fd);
    shm_unlink(name);
    return HG_ERR_ARG;
  }
  void* p = mmap(nullptr, L.bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  if (p == MAP_FAILED) {
    close(fd);
    shm_unlink(name);
    return HG_ERR_ARG;
  }
  s = new hg_service();
  s->cfg = cfg;
  s->name = name;
  s->fd = fd;
  s->v.base = static_cast<uint8_t*>(p);
  s->v.h = static_cast<Header*>(p);
  Header* h = s->v.h;  // a fresh object: zero-filled by ftruncate
  h->version = kVersion;
  h->nslots = cfg.slots;
  h->slot_words = slot_words;
  h->nchan = cfg.channels;
  h->bytes = L.bytes;
  h->slot_stride = L.slot_stride;
  h->off_slots = L.off_slots;
  h->off_chan = L.off_chan;
  h->off_rings = L.off_rings;
  h->off_free = L.off_free;
  h->off_queued = L.off_queued;
  h->nreg = nreg;
  h->flavor = flavor;
  std::atomic<uint64_t>* fb = s->v.free_bits();
  for (uint32_t w = 0; w < cfg.slots / 64; w++) fb[w].store(~0ull, std::memory_order_relaxed);
  s->tails.assign(cfg.channels, 0);
  s->touched.assign(cfg.channels, 0);
  s->released.assign(cfg.channels, 0);
  s->adopted.assign(cfg.channels, 0);
  s->outstanding.assign(cfg.channels, 0);
  s->owed_chan.assign(cfg.slots, hg_service::kNone);
  s->owed_gen.assign(cfg.slots, 0);
  s->lanes.resize(cfg.lanes);
#ifdef HG_SERVICE_TESTING
  if (const char* e = getenv("HG_SERVICE_TEST_FINISH_US")) s->test_finish_us = (uint32_t)atoi(e);
#endif
  return HG_OK;
}

void start(hg_service* s) {
  Header* h = s->v.h;
  h->state.store(kRunning, std::memory_order_release);
  std::atomic_thread_fence(std::memory_order_seq_cst);
  h->magic = kMagic;  // clients attach only once this is set
  s->th = std::thread([s] { s->run(); });
}

}  // namespace

extern "C" {

void hg_service_config_init(hg_service_config* c) {
  if (!c) return;
  c->slots = 8192;
  c->slot_bits = 0;
  c->channels = 256;
  c->lanes = 8;
  c->max_batch = 4096;
  c->max_wait_us = 50;
  c->quiet_us = 0;
  c->follow = 1;
  c->prepare = 1;
  c->overlap = 1;
}

int hg_service_create(hg_ctx* ctx, const char* name, const hg_service_config* cfg, hg_service** out) {
  if (!ctx) return HG_ERR_ARG;
  const size_t nreg = hg_registry_size(ctx);
  if (nreg == 0 || nreg > UINT32_MAX) return HG_ERR_ARG;
  hg_service* s = nullptr;
  int rc = create_common(name, cfg, (uint32_t)nreg, (uint32_t)hg_context_flavor(ctx), out, s);
  if (rc) return rc;
  GpuExec* g = new GpuExec(ctx);
  const size_t max_words = (size_t)s->cfg.max_batch * s->v.h->slot_words;
  // HG_SERVICE_PAD=0: unpadded lanes (the 12-lane split pairing, two waves of
  // different batches per SIMD) instead of the padded 16-lane kernel (one wave
  // per SIMD: the latency form); an A/B knob (tools/gpu_service_pad.sh)
  const char* pe = getenv("HG_SERVICE_PAD");
  const bool pad = !pe || atoi(pe) != 0;
  for (uint32_t i = 0; i < s->cfg.lanes; i++) {
    hg_lane* l = nullptr;
    rc = hg_lane_create(ctx, s->cfg.max_batch, max_words, s->cfg.overlap, &l);
    if (rc == HG_OK && !pad) rc = hg_lane_set_pairing_padding(l, 0);
    if (l) g->ln.push_back(l);
    if (rc) break;
  }
  if (rc) {
    delete g;
    munmap(s->v.base, s->v.h->bytes);
    close(s->fd);
    shm_unlink(name);
    delete s;
    return rc;
  }
  g->simd_count = hg_context_simds(ctx);
  if (const char* e = getenv("HG_SERVICE_W2")) s->w2_policy = atoi(e) != 0;
  s->ex = g;
  g->warm_up();  // under the context's current message, if it has one
  start(s);
  *out = s;
  return HG_OK;
}

int hg_service_create_echo(const char* name, const hg_service_config* cfg, uint32_t nreg, uint32_t delay_us,
                           hg_service** out) {
  if (nreg == 0) return HG_ERR_ARG;
  hg_service* s = nullptr;
  int rc = create_common(name, cfg, nreg, 0, out, s);
  if (rc) return rc;
  s->ex = new EchoExec((int)s->cfg.lanes, s->cfg.max_batch, (size_t)s->cfg.max_batch * s->v.h->slot_words, nreg,
                       delay_us);
  start(s);
  *out = s;
  return HG_OK;
}

void hg_service_destroy(hg_service* s) {
  if (!s) return;
  Header* h = s->v.h;
  h->state.store(kStopping, std::memory_order_seq_cst);
  s->stop.store(true, std::memory_order_release);
  h->doorbell.fetch_add(1, std::memory_order_seq_cst);
  futex_wake(&h->doorbell);
  s->th.join();  // what was queued is verified first
  h->state.store(kStopped, std::memory_order_seq_cst);
  // requests queued after the last look fail; every sleeper wakes and sees kStopped
  s->pending.clear();
  (void)s->intake();
  std::vector<Pending> ids(s->pending.begin(), s->pending.end());
  s->finish_slots(ids.data(), ids.size(), nullptr, HG_ERR_DEVICE);
  for (uint32_t c = 0; c < h->nchan; c++) {
    s->v.chan(c)->tail.fetch_add(0, std::memory_order_seq_cst);
    futex_wake(&s->v.chan(c)->tail);
  }
  delete s->ex;
  shm_unlink(s->name.c_str());
  munmap(s->v.base, h->bytes);
  close(s->fd);
  delete s;
}

int hg_service_stats(hg_service* s, uint64_t* batches, uint64_t* requests, uint64_t* max_in_flight) {
  if (!s) return HG_ERR_ARG;
  if (batches) *batches = s->v.h->batches.load();
  if (requests) *requests = s->v.h->requests.load();
  if (max_in_flight) *max_in_flight = s->max_in_flight;
  return HG_OK;
}

}  // extern "C"
