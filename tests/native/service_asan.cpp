// service_asan.cpp — CPU-only AddressSanitizer harness of the verifier
// service's trust boundary (hg_service.cpp + hg_client.cpp, the echo
// executor; no GPU, no HIP runtime). Built by tests/test_service.py with
//   g++ -fsanitize=address -g hg_service.cpp hg_client.cpp service_asan.cpp
// Client processes share the request slots with the GPU-owning process, so a
// buggy or hostile client can rewrite a slot after queuing it. The service
// must still never read or write outside its own buffers (processing.go:
// 342-352: a bitset that does not fit its level is an error, never a crash).
//
// Scenarios (exit 0 = every check held; ASan aborts on any bad access):
//   rewrite  a queued request's bitlen / level_size rewritten to the maximum
//            and to 2^32-1 while the dispatcher holds it: snapshot verdicts
//   orphan   a handle closed with tickets in flight: slots return, the
//            channel stays reserved until then, the next handle sees only
//            its own tickets
//   hostile  4 submitting threads while a fifth rewrites the size fields of
//            random slot headers continuously: every ticket comes back (its
//            code may be anything), no bad access
//   race     a handle closed while the batch holding its last tickets is
//            being finished (one channel, many rounds at random moments): the
//            channel is released only once the service holds none of its
//            slots, and every later handle sees exactly its own tickets
//   forged   an orphan header forged in shared memory (head far behind the
//            tail, ring entries naming another channel's finished slots):
//            the dispatcher neither stalls nor frees the other channel's
//            slots, whose owner still collects its verdicts
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <random>
#include <set>
#include <thread>
#include <vector>

#include "../../handel_amd/csrc/hg_shm.h"
#include "../../include/handel_client.h"
#include "../../include/handel_gpu.h"

// The GPU entry points hg_service.cpp references (GpuExec): never called by
// the echo executor; present so the service links without the HIP library.
extern "C" {
size_t hg_registry_size(hg_ctx*) { return 0; }
int hg_context_flavor(hg_ctx*) { return 0; }
int hg_context_simds(hg_ctx*) { return 0; }
int hg_set_message(hg_ctx*, const uint8_t*, size_t) { return HG_ERR_DEVICE; }
int hg_prepare_aggregate_msg(hg_ctx*, const uint8_t*, size_t) { return HG_ERR_DEVICE; }
int hg_prepare_aggregate_level(hg_ctx*, int) { return HG_ERR_DEVICE; }
int hg_lane_create(hg_ctx*, size_t, size_t, int, hg_lane**) { return HG_ERR_DEVICE; }
void hg_lane_destroy(hg_lane*) {}
int hg_lane_stage(hg_lane*, size_t, size_t, hg_request**, uint8_t**, uint64_t**) { return HG_ERR_DEVICE; }
int hg_lane_submit(hg_lane*) { return HG_ERR_DEVICE; }
int hg_lane_query(hg_lane*) { return -1; }
int hg_lane_wait(hg_lane*) { return HG_ERR_DEVICE; }
const int32_t* hg_lane_codes(hg_lane*) { return nullptr; }
int hg_lane_set_latency_form(hg_lane*, int) { return HG_ERR_DEVICE; }
int hg_lane_set_pairing_padding(hg_lane*, int) { return HG_ERR_DEVICE; }
}

using namespace hgshm;

static int failures = 0;
#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      fprintf(stderr, "%s:%d: check failed: %s\n", __FILE__, __LINE__, #c); \
      failures++;                                                  \
    }                                                              \
  } while (0)

static const uint8_t kMsg[] = "asan harness";

// the echo rule's signature: sig[0] = tampered, sig[1..8] = XOR of the words
static void echo_sig(const uint64_t* w, uint32_t nw, bool bad, uint8_t sig[64]) {
  uint64_t x = 0;
  for (uint32_t i = 0; i < nw; i++) x ^= w[i];
  memset(sig, 0, 64);
  sig[0] = bad ? 1 : 0;
  memcpy(sig + 1, &x, 8);
}

struct Region {
  uint8_t* base = nullptr;
  size_t bytes = 0;
  View v;
  explicit Region(const char* name) {
    const int fd = shm_open(name, O_RDWR, 0);
    struct stat st;
    fstat(fd, &st);
    bytes = (size_t)st.st_size;
    base = static_cast<uint8_t*>(mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0));
    close(fd);
    v.base = base;
    v.h = reinterpret_cast<Header*>(base);
  }
  ~Region() { munmap(base, bytes); }
};

static hg_service* echo(const char* name, uint32_t lanes, uint32_t channels, uint32_t slots, uint32_t wait_us,
                        int follow, uint32_t nreg, uint32_t delay_us) {
  hg_service_config cfg;
  hg_service_config_init(&cfg);
  cfg.lanes = lanes;
  cfg.channels = channels;
  cfg.slots = slots;
  cfg.max_wait_us = wait_us;
  cfg.follow = follow;
  hg_service* s = nullptr;
  if (hg_service_create_echo(name, &cfg, nreg, delay_us, &s) != HG_OK) return nullptr;
  return s;
}

static void scenario_rewrite(const char* name) {
  hg_service* s = echo(name, 1, 4, 64, 300000, 0, 256, 10);
  CHECK(s);
  if (!s) return;
  hg_client* c = nullptr;
  CHECK(hg_client_open(name, &c) == HG_OK);
  Region r(name);
  const uint32_t bigs[2] = {r.v.h->slot_words * 64u, 0xFFFFFFFFu};
  for (uint32_t big : bigs) {
    uint64_t w[1] = {0x0123456789abcdefull};
    uint8_t sig[64];
    echo_sig(w, 1, false, sig);
    hg_request q{64, 64, 64, 0};
    uint64_t t = 0;
    CHECK(hg_client_submit(c, kMsg, sizeof kMsg, &q, w, sig, &t) == HG_OK);
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
    Slot* sl = r.v.slot((uint32_t)t);
    CHECK(sl->state.load() == kSlotTaken);
    sl->offset = 0;
    sl->bitlen = big;
    sl->level_size = big;
    int32_t code = -1;
    CHECK(hg_client_wait(c, t, &code) == HG_OK);
    CHECK(code == HG_OK);
  }
  hg_client_close(c);
  hg_service_destroy(s);
}

static void scenario_orphan(const char* name) {
  hg_service* s = echo(name, 1, 1, 64, 10, 1, 128, 150000);
  CHECK(s);
  if (!s) return;
  hg_client* a = nullptr;
  CHECK(hg_client_open(name, &a) == HG_OK);
  uint64_t w[1] = {1};
  uint8_t sig[64];
  echo_sig(w, 1, false, sig);
  hg_request q{0, 64, 64, 0};
  for (int i = 0; i < 10; i++) {
    uint64_t t;
    CHECK(hg_client_submit(a, kMsg, sizeof kMsg, &q, w, sig, &t) == HG_OK);
  }
  hg_client_close(a);
  hg_client* b = nullptr;
  CHECK(hg_client_open(name, &b) != HG_OK);  // reserved while the ten run
  const auto t0 = std::chrono::steady_clock::now();
  while (hg_client_open(name, &b) != HG_OK) {
    if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(5)) {
      CHECK(!"orphaned channel never released");
      hg_service_destroy(s);
      return;
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(5));
  }
  std::set<uint64_t> mine;
  for (int i = 0; i < 64; i++) {  // every slot of the region
    uint64_t t;
    CHECK(hg_client_submit(b, kMsg, sizeof kMsg, &q, w, sig, &t) == HG_OK);
    mine.insert(t);
  }
  std::set<uint64_t> got;
  uint64_t tk[64];
  int32_t cd[64];
  while (got.size() < mine.size()) {
    const int n = hg_client_wait_any(b, tk, cd, 64, 2000000);
    CHECK(n > 0);
    if (n <= 0) break;
    for (int i = 0; i < n; i++) {
      CHECK(mine.count(tk[i]) == 1);
      CHECK(got.insert(tk[i]).second);
      CHECK(cd[i] == HG_OK);
    }
  }
  hg_client_close(b);
  hg_service_destroy(s);
}

static void scenario_hostile(const char* name) {
  const uint32_t nreg = 1000;
  hg_service* s = echo(name, 4, 8, 256, 50, 1, nreg, 30);
  CHECK(s);
  if (!s) return;
  hg_client* c = nullptr;
  CHECK(hg_client_open(name, &c) == HG_OK);
  Region r(name);
  std::atomic<bool> stop{false};
  std::thread evil([&] {
    std::mt19937_64 g(7);
    while (!stop.load()) {
      Slot* sl = r.v.slot((uint32_t)(g() % r.v.h->nslots));
      const uint32_t pick[4] = {0, r.v.h->slot_words * 64u, 0xFFFFFFFFu, (uint32_t)g()};
      sl->bitlen = pick[g() % 4];
      sl->level_size = pick[g() % 4];
      sl->offset = pick[g() % 4];
    }
  });
  std::vector<std::thread> th;
  std::atomic<int> answered{0}, lost{0};
  for (int k = 0; k < 4; k++)
    th.emplace_back([&, k] {
      std::mt19937_64 g(100 + k);
      std::vector<uint64_t> w(16);
      for (int i = 0; i < 200; i++) {
        const uint32_t bits = 1 + (uint32_t)(g() % nreg);
        for (auto& x : w) x = g();
        uint8_t sig[64];
        echo_sig(w.data(), (bits + 63) / 64, false, sig);
        hg_request q{0, bits, bits, 0};
        uint64_t t;
        if (hg_client_submit(c, kMsg, sizeof kMsg, &q, w.data(), sig, &t) != HG_OK) continue;
        int32_t code;
        if (hg_client_wait(c, t, &code) == HG_OK) answered++;
        else lost++;
      }
    });
  for (auto& t : th) t.join();
  stop = true;
  evil.join();
  CHECK(answered.load() == 800 && lost.load() == 0);
  hg_client_close(c);
  hg_service_destroy(s);
}

static void scenario_race(const char* name) {
  // one channel, so every round's handle reuses the channel the previous one
  // closed; the dispatcher pauses 100 us after each completion it pushes
  // (HG_SERVICE_TEST_FINISH_US), so a close lands between a batch's pushes
  // and the publication of its tail in many rounds
  setenv("HG_SERVICE_TEST_FINISH_US", "100", 1);
  hg_service* s = echo(name, 2, 1, 128, 20, 0, 128, 300);
  unsetenv("HG_SERVICE_TEST_FINISH_US");
  CHECK(s);
  if (!s) return;
  std::mt19937_64 g(11);
  uint64_t w[1] = {3};
  uint8_t sig[64];
  echo_sig(w, 1, false, sig);
  hg_request q{0, 64, 64, 0};
  for (int round = 0; round < 300; round++) {
    hg_client* c = nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    while (hg_client_open(name, &c) != HG_OK) {
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(5)) {
        CHECK(!"channel never released");
        hg_service_destroy(s);
        return;
      }
      std::this_thread::yield();
    }
    // the previous handles' tickets never show up here: collect this
    // handle's first ticket and nothing else
    uint64_t t = 0;
    CHECK(hg_client_submit(c, kMsg, sizeof kMsg, &q, w, sig, &t) == HG_OK);
    uint64_t tk[8];
    int32_t cd[8];
    const int n = hg_client_wait_any(c, tk, cd, 8, 2000000);
    CHECK(n == 1 && tk[0] == t && cd[0] == HG_OK);
    // then several more, and close at a random moment around their batch
    const int k = 1 + (int)(g() % 6);
    for (int i = 0; i < k; i++) CHECK(hg_client_submit(c, kMsg, sizeof kMsg, &q, w, sig, &t) == HG_OK);
    std::this_thread::sleep_for(std::chrono::microseconds(g() % 1200));
    hg_client_close(c);
  }
  // every slot comes back: a fresh handle claims the whole region
  hg_client* c = nullptr;
  const auto t0 = std::chrono::steady_clock::now();
  while (hg_client_open(name, &c) != HG_OK && std::chrono::steady_clock::now() - t0 < std::chrono::seconds(5))
    std::this_thread::sleep_for(std::chrono::milliseconds(1));
  CHECK(c);
  if (c) {
    std::set<uint64_t> mine, got;
    for (int i = 0; i < 128; i++) {
      uint64_t t;
      CHECK(hg_client_submit(c, kMsg, sizeof kMsg, &q, w, sig, &t) == HG_OK);
      mine.insert(t);
    }
    uint64_t tk[128];
    int32_t cd[128];
    while (got.size() < mine.size()) {
      const int n = hg_client_wait_any(c, tk, cd, 128, 2000000);
      CHECK(n > 0);
      if (n <= 0) break;
      for (int i = 0; i < n; i++) CHECK(mine.count(tk[i]) == 1 && got.insert(tk[i]).second);
    }
    hg_client_close(c);
  }
  hg_service_destroy(s);
}

static void scenario_forged(const char* name) {
  hg_service* s = echo(name, 2, 4, 64, 20, 0, 128, 200);
  CHECK(s);
  if (!s) return;
  hg_client* victim = nullptr;
  hg_client* other = nullptr;
  CHECK(hg_client_open(name, &victim) == HG_OK);  // channel 0
  CHECK(hg_client_open(name, &other) == HG_OK);   // channel 1
  Region r(name);
  uint64_t w[1] = {5};
  uint8_t sig[64];
  echo_sig(w, 1, false, sig);
  hg_request q{0, 64, 64, 0};
  // the victim's tickets finish but stay uncollected
  std::vector<uint64_t> vt(8);
  for (auto& t : vt) CHECK(hg_client_submit(victim, kMsg, sizeof kMsg, &q, w, sig, &t) == HG_OK);
  const auto t0 = std::chrono::steady_clock::now();
  while (r.v.chan(0)->tail.load() < 8 && std::chrono::steady_clock::now() - t0 < std::chrono::seconds(5))
    std::this_thread::sleep_for(std::chrono::milliseconds(1));
  CHECK(r.v.chan(0)->tail.load() == 8);
  // a hostile process forges channel 2 as orphaned: (a) a head ~2^32
  // positions behind the tail, (b) then ring entries naming the victim's
  // finished slots
  Channel* f = r.v.chan(2);
  f->used.store(kChanOrphaned);
  f->head = f->tail.load() + 1;
  r.v.h->orphans.fetch_add(1);
  r.v.h->doorbell.fetch_add(1);
  std::this_thread::sleep_for(std::chrono::milliseconds(20));
  Channel* f3 = r.v.chan(3);
  uint32_t* ring3 = r.v.ring(3);
  for (int i = 0; i < 8; i++) ring3[i] = (uint32_t)vt[i];
  f3->head = 0;
  f3->tail.store(8);
  f3->used.store(kChanOrphaned);
  r.v.h->orphans.fetch_add(1);
  r.v.h->doorbell.fetch_add(1);
  std::this_thread::sleep_for(std::chrono::milliseconds(20));
  // the dispatcher still serves the other channel
  int32_t code = -1;
  uint64_t t;
  CHECK(hg_client_submit(other, kMsg, sizeof kMsg, &q, w, sig, &t) == HG_OK);
  CHECK(hg_client_wait(other, t, &code) == HG_OK && code == HG_OK);
  // and the victim's slots were not freed under it: its verdicts are there
  for (uint64_t x : vt) {
    CHECK((uint32_t)(x >> 32) == r.v.slot((uint32_t)x)->gen);
    code = -1;
    CHECK(hg_client_wait(victim, x, &code) == HG_OK && code == HG_OK);
  }
  hg_client_close(victim);
  hg_client_close(other);
  hg_service_destroy(s);
}

int main(int argc, char** argv) {
  char name[96];
  const char* only = argc > 1 ? argv[1] : "";
  if (!*only || !strcmp(only, "rewrite")) {
    snprintf(name, sizeof name, "/hg_asan_rw_%d", (int)getpid());
    scenario_rewrite(name);
  }
  if (!*only || !strcmp(only, "orphan")) {
    snprintf(name, sizeof name, "/hg_asan_or_%d", (int)getpid());
    scenario_orphan(name);
  }
  if (!*only || !strcmp(only, "hostile")) {
    snprintf(name, sizeof name, "/hg_asan_ho_%d", (int)getpid());
    scenario_hostile(name);
  }
  if (!*only || !strcmp(only, "race")) {
    snprintf(name, sizeof name, "/hg_asan_ra_%d", (int)getpid());
    scenario_race(name);
  }
  if (!*only || !strcmp(only, "forged")) {
    snprintf(name, sizeof name, "/hg_asan_fo_%d", (int)getpid());
    scenario_forged(name);
  }
  printf("{\"failures\": %d}\n", failures);
  return failures ? 1 : 0;
}
