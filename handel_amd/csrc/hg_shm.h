// hg_shm.h — shared-memory layout of the verifier service.
//
// One GPU-owning process (hg_service.cpp, in libhandel_gpu.so) serves the
// aggregate checks of many client processes (hg_client.cpp, in
// libhandel_client.so, which never touches the GPU): simul's P processes of
// k Handel instances each (simul/node/main.go:63-131), every instance's
// processLoop checking one multisignature at a time (processing.go:228-287).
// The region is a POSIX shared-memory object (shm_open name):
//
//   Header | Slot[nslots] | Channel[nchan] | ring[nchan][nslots] u32 |
//   free bitmap[nslots/64] | queued bitmap[nslots/64]
//
// A request lives in a slot: the client claims a free slot (free bitmap),
// writes the request, its bitset words and signature, marks it queued
// (queued bitmap) and rings the doorbell if the server sleeps. The server
// takes queued slots into GPU batches, writes each code into its slot and
// pushes the slot id into the ring of the slot's channel (one channel per
// client handle), waking the channel's sleepers once per batch. The client
// copies the code out and frees the slot. Every cross-process handoff is one
// atomic with release/acquire order; sleeps are futexes on shared words.
#pragma once
#include <linux/futex.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <climits>
#include <cstddef>
#include <cstdint>

#include "../../include/handel_gpu.h"

namespace hgshm {

constexpr uint64_t kMagic = 0x3130435653474855ull;  // "UHGSVC01"
constexpr uint32_t kVersion = 2;
constexpr uint32_t kMaxMsgs = 32;   // distinct messages pinned at once
constexpr uint32_t kMsgCap = 1024;  // bytes of one message

enum : uint32_t { kSlotFree = 0, kSlotFilling = 1, kSlotQueued = 2, kSlotTaken = 3, kSlotDone = 4 };
enum : uint32_t { kRunning = 1, kStopping = 2, kStopped = 3 };
enum : uint32_t { kMsgEmpty = 0, kMsgBusy = 1, kMsgReady = 2 };
// Channel.used: free, held by a client handle, or orphaned (its handle closed
// with requests in flight: the service frees those slots itself and releases
// the channel once none is left, so no later handle sees foreign completions)
enum : uint32_t { kChanFree = 0, kChanUsed = 1, kChanOrphaned = 2 };

static_assert(sizeof(std::atomic<uint32_t>) == 4 && sizeof(std::atomic<uint64_t>) == 8, "lock-free shared words");

struct alignas(64) Slot {
  std::atomic<uint32_t> state;
  uint32_t gen;  // bumped by every claim; a ticket is (gen << 32) | slot
  uint32_t chan;
  uint32_t msg, msg_gen;
  int32_t code;
  uint32_t offset, bitlen, level_size;
  uint32_t pad[7];
  uint8_t sig[64];
  // uint64_t words[slot_words] follow (the slot stride)
  uint64_t* words() { return reinterpret_cast<uint64_t*>(this + 1); }
};
static_assert(sizeof(Slot) == 128, "slot header");

struct alignas(64) Channel {
  std::atomic<uint32_t> used;      // kChanFree / kChanUsed / kChanOrphaned
  std::atomic<uint32_t> tail;      // completions pushed so far (futex word)
  std::atomic<uint32_t> waiters;   // client threads asleep on tail
  uint32_t pid;
  std::atomic<uint32_t> inflight;  // slots of this channel claimed and not yet freed
  uint32_t head;                   // the closing handle's ring position (valid once orphaned)
};
static_assert(sizeof(Channel) == 64, "channel");

struct alignas(64) Msg {
  std::atomic<uint32_t> state;  // kMsgEmpty / kMsgBusy (being written) / kMsgReady
  std::atomic<uint32_t> refs;   // client handles holding it
  uint32_t gen;                 // bumped when the entry is rewritten
  uint32_t len;
  uint8_t bytes[kMsgCap];
};

struct alignas(64) Header {
  uint64_t magic;
  uint32_t version, nslots, slot_words, nchan;
  uint64_t bytes, slot_stride, off_slots, off_chan, off_rings, off_free, off_queued;
  uint32_t nreg, flavor;
  alignas(64) std::atomic<uint32_t> state;
  alignas(64) std::atomic<uint32_t> doorbell;  // futex word: clients bump it while the server sleeps
  std::atomic<uint32_t> sleeping;
  alignas(64) std::atomic<uint32_t> msg_lock;  // guards msgs[] rewrites (rare)
  alignas(64) std::atomic<uint64_t> batches, requests;
  std::atomic<uint32_t> orphans;  // bumped by every handle closed with requests in flight
  Msg msgs[kMaxMsgs];
};

struct Layout {
  uint64_t bytes, slot_stride, off_slots, off_chan, off_rings, off_free, off_queued;
};
inline uint64_t align64(uint64_t x) { return (x + 63) & ~(uint64_t)63; }
inline Layout layout(uint32_t nslots, uint32_t slot_words, uint32_t nchan) {
  Layout L;
  L.slot_stride = align64(sizeof(Slot) + 8ull * slot_words);
  L.off_slots = align64(sizeof(Header));
  L.off_chan = L.off_slots + L.slot_stride * nslots;
  L.off_rings = align64(L.off_chan + sizeof(Channel) * (uint64_t)nchan);
  L.off_free = align64(L.off_rings + 4ull * nslots * nchan);
  L.off_queued = L.off_free + 8ull * (nslots / 64);
  L.bytes = align64(L.off_queued + 8ull * (nslots / 64));
  return L;
}

struct View {
  Header* h = nullptr;
  uint8_t* base = nullptr;
  Slot* slot(uint32_t i) const { return reinterpret_cast<Slot*>(base + h->off_slots + h->slot_stride * i); }
  Channel* chan(uint32_t c) const { return reinterpret_cast<Channel*>(base + h->off_chan) + c; }
  uint32_t* ring(uint32_t c) const {
    return reinterpret_cast<uint32_t*>(base + h->off_rings) + (uint64_t)c * h->nslots;
  }
  std::atomic<uint64_t>* free_bits() const { return reinterpret_cast<std::atomic<uint64_t>*>(base + h->off_free); }
  std::atomic<uint64_t>* queued_bits() const {
    return reinterpret_cast<std::atomic<uint64_t>*>(base + h->off_queued);
  }
};

// futexes on shared (non-private) words
inline void futex_wait(std::atomic<uint32_t>* w, uint32_t val, long timeout_us) {
  timespec ts{timeout_us / 1000000, (timeout_us % 1000000) * 1000};
  syscall(SYS_futex, reinterpret_cast<uint32_t*>(w), FUTEX_WAIT, val, timeout_us >= 0 ? &ts : nullptr, nullptr, 0);
}
inline void futex_wake(std::atomic<uint32_t>* w, int n = INT_MAX) {
  syscall(SYS_futex, reinterpret_cast<uint32_t*>(w), FUTEX_WAKE, n, nullptr, nullptr, 0);
}
inline void cpu_relax() { __builtin_ia32_pause(); }

}  // namespace hgshm
