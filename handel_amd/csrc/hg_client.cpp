// hg_client.cpp — client side of the verifier service (include/handel_client.h;
// layout and protocol in hg_shm.h). Built into libhandel_client.so with the
// host compiler only: a simul process (simul/node/main.go:63-131) links it
// instead of opening a GPU context, and hands each Handel instance's
// verifySignature (processing.go:342-368) to the one process that owns the GPU.
#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>

#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/handel_client.h"
#include "hg_codes.h"
#include "hg_shm.h"

using namespace hgshm;

namespace {
struct Pinned {
  std::string bytes;
  uint32_t id, gen;
  uint64_t outstanding;  // this handle's requests under it not yet drained
};
}  // namespace

struct hg_client {
  View v;
  size_t bytes = 0;
  uint32_t ch = 0;
  Channel* chan = nullptr;
  uint32_t hint = 0;  // where the next slot search starts
  std::mutex mu;      // guards everything below
  std::vector<Pinned> pinned;  // this handle's message references (refs held)
  uint32_t head = 0;           // completions consumed from the channel ring
  std::unordered_map<uint64_t, int32_t> done;  // collected from the ring, not yet returned
  std::deque<uint64_t> order;                  // the same tickets, completion order
  bool draining = false;                       // one thread sleeps on the ring at a time
  std::condition_variable cv;
};

namespace {

// moves the channel's new completions into the handle (codes copied, slots freed)
void drain_locked(hg_client* c) {
  const uint32_t tail = c->chan->tail.load(std::memory_order_acquire);
  const uint32_t* ring = c->v.ring(c->ch);
  const uint32_t cap = c->v.h->nslots;
  std::atomic<uint64_t>* fb = c->v.free_bits();
  while (c->head != tail) {
    const uint32_t id = ring[c->head % cap];
    c->head++;
    Slot* s = c->v.slot(id);
    if (s->state.load(std::memory_order_acquire) != kSlotDone) continue;
    for (Pinned& p : c->pinned)
      if (p.id == s->msg && p.gen == s->msg_gen && p.outstanding) {
        p.outstanding--;
        break;
      }
    const uint64_t t = ((uint64_t)s->gen << 32) | id;
    c->done[t] = s->code;
    c->order.push_back(t);
    s->state.store(kSlotFree, std::memory_order_release);
    fb[id / 64].fetch_or(1ull << (id % 64), std::memory_order_release);
    c->chan->inflight.fetch_sub(1, std::memory_order_acq_rel);
  }
}

bool stopped(const hg_client* c) { return c->v.h->state.load(std::memory_order_acquire) == kStopped; }

// sleeps until the ring moves past `seen`, the deadline passes or the service
// stops (the caller re-checks); spins briefly first: completions come in
// bursts a few hundred microseconds apart
void sleep_on_ring(hg_client* c, uint32_t seen, long timeout_us) {
  for (int i = 0; i < 4000; i++) {
    if (c->chan->tail.load(std::memory_order_acquire) != seen || stopped(c)) return;
    cpu_relax();
  }
  c->chan->waiters.fetch_add(1, std::memory_order_seq_cst);
  if (c->chan->tail.load(std::memory_order_seq_cst) == seen && !stopped(c))
    futex_wait(&c->chan->tail, seen, timeout_us < 0 || timeout_us > 100000 ? 100000 : timeout_us);
  c->chan->waiters.fetch_sub(1, std::memory_order_seq_cst);
}

// a message entry this handle holds a reference to (claimed or added); the
// caller counts the request it submits under it (outstanding)
Pinned* pin_message(hg_client* c, const uint8_t* msg, size_t len) {
  for (Pinned& p : c->pinned)
    if (p.bytes.size() == len && (len == 0 || memcmp(p.bytes.data(), msg, len) == 0)) return &p;
  // at most 4 messages per handle: drop a reference no queued request uses
  if (c->pinned.size() >= 4) {
    drain_locked(c);
    size_t k = 0;
    while (k < c->pinned.size() && c->pinned[k].outstanding) k++;
    if (k == c->pinned.size()) return nullptr;
    c->v.h->msgs[c->pinned[k].id].refs.fetch_sub(1, std::memory_order_acq_rel);
    c->pinned.erase(c->pinned.begin() + (long)k);
  }
  uint32_t idv = 0, genv = 0;
  uint32_t* id = &idv;
  uint32_t* gen = &genv;
  Header* h = c->v.h;
  while (h->msg_lock.exchange(1, std::memory_order_acquire)) sched_yield();
  int found = -1, empty = -1;
  for (uint32_t i = 0; i < kMaxMsgs; i++) {
    Msg& m = h->msgs[i];
    const uint32_t st = m.state.load(std::memory_order_acquire);
    if (st == kMsgReady && m.len == len && (len == 0 || memcmp(m.bytes, msg, len) == 0)) {
      found = (int)i;
      break;
    }
    if (empty < 0 && (st == kMsgEmpty || (st == kMsgReady && m.refs.load() == 0))) empty = (int)i;
  }
  int rc = HG_OK;
  if (found < 0 && empty >= 0) {
    Msg& m = h->msgs[empty];
    m.state.store(kMsgBusy, std::memory_order_relaxed);
    m.gen++;
    m.len = (uint32_t)len;
    if (len) memcpy(m.bytes, msg, len);
    m.state.store(kMsgReady, std::memory_order_release);
    found = empty;
  }
  if (found >= 0) {
    h->msgs[found].refs.fetch_add(1, std::memory_order_acq_rel);
    *id = (uint32_t)found;
    *gen = h->msgs[found].gen;
  } else {
    rc = HG_ERR_ARG;  // every entry is held by some client
  }
  h->msg_lock.store(0, std::memory_order_release);
  if (rc != HG_OK) return nullptr;
  c->pinned.push_back(Pinned{std::string(reinterpret_cast<const char*>(msg), len), *id, *gen, 0});
  return &c->pinned.back();
}

// claims a free slot; -1 if none frees up within ~2 s
int64_t claim_slot(hg_client* c) {
  std::atomic<uint64_t>* fb = c->v.free_bits();
  const uint32_t words = c->v.h->nslots / 64;
  const auto t0 = std::chrono::steady_clock::now();
  for (int round = 0;; round++) {
    for (uint32_t k = 0; k < words; k++) {
      const uint32_t w = (c->hint + k) % words;
      uint64_t x = fb[w].load(std::memory_order_relaxed);
      while (x) {
        const uint64_t bit = x & (~x + 1);
        if (fb[w].compare_exchange_weak(x, x & ~bit, std::memory_order_acq_rel, std::memory_order_relaxed)) {
          c->hint = w;
          return (int64_t)w * 64 + __builtin_ctzll(bit);
        }
      }
    }
    if (c->v.h->state.load(std::memory_order_acquire) != kRunning) return -1;
    if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) return -1;
    sched_yield();
  }
}

}  // namespace

extern "C" {

int hg_client_open(const char* name, hg_client** out) {
  if (!name || !out) return HG_ERR_ARG;
  *out = nullptr;
  const int fd = shm_open(name, O_RDWR, 0);
  if (fd < 0) return HG_ERR_ARG;
  struct stat st;
  if (fstat(fd, &st) != 0 || (size_t)st.st_size < sizeof(Header)) {
    close(fd);
    return HG_ERR_ARG;
  }
  void* p = mmap(nullptr, (size_t)st.st_size, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) return HG_ERR_ARG;
  Header* h = static_cast<Header*>(p);
  const bool ok = h->magic == kMagic && h->version == kVersion && h->bytes == (uint64_t)st.st_size &&
                  h->state.load(std::memory_order_acquire) == kRunning && h->nslots % 64 == 0;
  if (!ok) {
    munmap(p, (size_t)st.st_size);
    return HG_ERR_ARG;
  }
  hg_client* c = new hg_client();
  c->v.h = h;
  c->v.base = static_cast<uint8_t*>(p);
  c->bytes = (size_t)st.st_size;
  bool got = false;
  for (uint32_t i = 0; i < h->nchan && !got; i++) {
    uint32_t z = 0;
    if (c->v.chan(i)->used.compare_exchange_strong(z, 1, std::memory_order_acq_rel)) {
      c->ch = i;
      got = true;
    }
  }
  if (!got) {
    munmap(p, c->bytes);
    delete c;
    return HG_ERR_ARG;
  }
  c->chan = c->v.chan(c->ch);
  // (a released channel owns no slot: inflight is 0)
  c->chan->pid = (uint32_t)getpid();
  c->head = c->chan->tail.load(std::memory_order_acquire);
  c->hint = (uint32_t)(c->ch * 7) % (h->nslots / 64);
  *out = c;
  return HG_OK;
}

void hg_client_close(hg_client* c) {
  if (!c) return;
  {
    std::lock_guard<std::mutex> g(c->mu);
    drain_locked(c);  // frees the slots of finished, uncollected tickets
    for (const Pinned& p : c->pinned) c->v.h->msgs[p.id].refs.fetch_sub(1, std::memory_order_acq_rel);
    c->pinned.clear();
    if (c->chan->inflight.load(std::memory_order_acquire) == 0) {
      c->chan->used.store(kChanFree, std::memory_order_release);
    } else {
      // tickets still in flight: the channel stays reserved (a new handle
      // would otherwise collect their completions) and the service frees
      // their slots itself, from where this handle's drain stopped
      Header* h = c->v.h;
      c->chan->head = c->head;
      c->chan->used.store(kChanOrphaned, std::memory_order_seq_cst);
      h->orphans.fetch_add(1, std::memory_order_seq_cst);
      if (h->sleeping.load(std::memory_order_seq_cst)) {
        h->doorbell.fetch_add(1, std::memory_order_seq_cst);
        futex_wake(&h->doorbell, 1);
      }
    }
  }
  munmap(c->v.base, c->bytes);
  delete c;
}

int hg_client_submit(hg_client* c, const uint8_t* msg, size_t len, const hg_request* req, const uint64_t* words,
                     const uint8_t* sig, uint64_t* ticket) {
  if (!c || !req || !sig || !ticket || (!msg && len) || len > kMsgCap) return HG_ERR_ARG;
  Header* h = c->v.h;
  const uint32_t nw = (req->bitlen + 63) / 64;
  if (req->bitlen > h->slot_words * 64u || (nw && !words)) return HG_ERR_ARG;
  if (h->state.load(std::memory_order_acquire) != kRunning) return HG_ERR_ARG;
  uint32_t mid, mgen;
  {
    std::lock_guard<std::mutex> g(c->mu);
    Pinned* p = pin_message(c, msg, len);
    if (!p) return HG_ERR_ARG;
    mid = p->id;
    mgen = p->gen;
    p->outstanding++;
  }
  c->chan->inflight.fetch_add(1, std::memory_order_acq_rel);  // before the slot can complete
  const int64_t id = claim_slot(c);
  if (id < 0) {
    c->chan->inflight.fetch_sub(1, std::memory_order_acq_rel);
    std::lock_guard<std::mutex> g(c->mu);
    for (Pinned& p : c->pinned)
      if (p.id == mid && p.gen == mgen && p.outstanding) p.outstanding--;
    return HG_ERR_ARG;
  }
  Slot* s = c->v.slot((uint32_t)id);
  s->state.store(kSlotFilling, std::memory_order_relaxed);
  s->gen++;
  s->chan = c->ch;
  s->msg = mid;
  s->msg_gen = mgen;
  s->code = -1;
  s->offset = req->offset;
  s->bitlen = req->bitlen;
  s->level_size = req->level_size;
  memcpy(s->sig, sig, 64);
  if (nw) memcpy(s->words(), words, 8ull * nw);
  const uint64_t t = ((uint64_t)s->gen << 32) | (uint64_t)id;
  s->state.store(kSlotQueued, std::memory_order_release);
  c->v.queued_bits()[id / 64].fetch_or(1ull << (id % 64), std::memory_order_seq_cst);
  if (h->sleeping.load(std::memory_order_seq_cst)) {
    h->doorbell.fetch_add(1, std::memory_order_seq_cst);
    futex_wake(&h->doorbell, 1);
  }
  *ticket = t;
  return HG_OK;
}

int hg_client_wait_any(hg_client* c, uint64_t* tickets, int32_t* codes, size_t cap, long timeout_us) {
  if (!c || !tickets || !codes || cap == 0) return -HG_ERR_ARG;
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::microseconds(timeout_us < 0 ? 0 : timeout_us);
  std::unique_lock<std::mutex> lk(c->mu);
  for (;;) {
    drain_locked(c);
    size_t k = 0;
    while (k < cap && !c->order.empty()) {
      const uint64_t t = c->order.front();
      c->order.pop_front();
      auto it = c->done.find(t);
      if (it == c->done.end()) continue;  // collected by hg_client_wait
      tickets[k] = t;
      codes[k] = it->second;
      c->done.erase(it);
      k++;
    }
    if (k) return (int)k;
    if (stopped(c)) {
      drain_locked(c);
      if (c->order.empty()) return -HG_ERR_DEVICE;
      continue;
    }
    long left = -1;
    if (timeout_us >= 0) {
      left = (long)std::chrono::duration_cast<std::chrono::microseconds>(deadline -
                                                                         std::chrono::steady_clock::now()).count();
      if (left <= 0) return 0;
    }
    if (c->draining) {
      if (left < 0) c->cv.wait(lk);
      else c->cv.wait_for(lk, std::chrono::microseconds(left));
      continue;
    }
    const uint32_t seen = c->head;
    c->draining = true;
    lk.unlock();
    sleep_on_ring(c, seen, left);
    lk.lock();
    c->draining = false;
    c->cv.notify_all();
  }
}

int hg_client_wait(hg_client* c, uint64_t t, int32_t* code) {
  if (!c) return HG_ERR_ARG;
  const uint32_t id = (uint32_t)t;
  if (id >= c->v.h->nslots) return HG_ERR_ARG;
  std::unique_lock<std::mutex> lk(c->mu);
  for (;;) {
    drain_locked(c);
    auto it = c->done.find(t);
    if (it != c->done.end()) {
      if (code) *code = it->second;
      c->done.erase(it);
      return HG_OK;
    }
    // a ticket of this handle still in flight (only this handle's drain frees its slots)
    const Slot* s = c->v.slot(id);
    const uint32_t st = s->state.load(std::memory_order_acquire);
    if (s->gen != (uint32_t)(t >> 32) || s->chan != c->ch || st == kSlotFree || st == kSlotFilling)
      return HG_ERR_ARG;
    if (stopped(c)) return HG_ERR_DEVICE;
    if (c->draining) {
      c->cv.wait_for(lk, std::chrono::milliseconds(100));
      continue;
    }
    const uint32_t seen = c->head;
    c->draining = true;
    lk.unlock();
    sleep_on_ring(c, seen, -1);
    lk.lock();
    c->draining = false;
    c->cv.notify_all();
  }
}

int hg_client_verify_aggregate(hg_client* c, const uint8_t* msg, size_t len, const hg_request* req,
                               const uint64_t* words, const uint8_t* sig, int32_t* code) {
  uint64_t t = 0;
  int rc = hg_client_submit(c, msg, len, req, words, sig, &t);
  if (rc) return rc;
  return hg_client_wait(c, t, code);
}

int hg_client_stats(hg_client* c, uint64_t* batches, uint64_t* requests) {
  if (!c) return HG_ERR_ARG;
  if (batches) *batches = c->v.h->batches.load(std::memory_order_relaxed);
  if (requests) *requests = c->v.h->requests.load(std::memory_order_relaxed);
  return HG_OK;
}

uint32_t hg_client_slot_bits(hg_client* c) { return c ? c->v.h->slot_words * 64u : 0; }

int hg_client_flavor(hg_client* c) { return c ? (int)c->v.h->flavor : -1; }

const char* hg_client_code_string(hg_client* c, int code) {
  return hg::code_text(code, c ? (int)c->v.h->flavor : HG_FLAVOR_GO);
}

const char* hg_client_processing_error_string(hg_client* c, int code) {
  return hg::processing_text(code, c ? (int)c->v.h->flavor : HG_FLAVOR_GO);
}

}  // extern "C"
