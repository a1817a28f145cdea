// hg_batcher.cpp — launch-merging request queue over one hg_ctx (C ABI in
// include/handel_gpu.h, hg_batcher_*).
//
// Handel's evaluator checks one signature at a time per instance
// (processing.go:228-287: processLoop -> readTodos -> verifyAndPublish ->
// verifySignature), and a simul process runs k instances concurrently
// (simul/node/main.go:63-131). Each instance's check becomes one request
// here; a dispatcher thread merges whatever is queued into ONE
// hg_verify_aggregate_msg batch (grouped by message, at most max_batch
// requests) and wakes every caller with its own code. While the GPU runs a
// batch the next one accumulates, so the batch width follows the load: one
// request when a single instance is active, hundreds when k instances are.
// An idle dispatcher lingers at most max_wait_us after the oldest queued
// request before launching a partial batch.
//
// Built only on the public C ABI: the batcher holds no device state of its
// own and the context's lock still serialises submissions from elsewhere.
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/handel_gpu.h"

// A ticket carries its own completion state: hg_batcher_wait touches only
// the ticket, so a wait may outlive the batcher (hg_batcher_destroy verifies
// every queued ticket before it returns).
struct hg_ticket {
  std::string msg;
  hg_request req{};
  std::vector<uint64_t> words;
  uint8_t sig[64];
  std::chrono::steady_clock::time_point t_submit;
  std::mutex mu;
  std::condition_variable cv;
  int32_t code = HG_OK;  // guarded by mu
  int rc = HG_OK;
  bool done = false;
};

struct hg_batcher {
  hg_ctx* ctx = nullptr;
  size_t max_batch = 4096;
  std::chrono::microseconds max_wait{200};
  std::mutex mu;
  std::condition_variable cv_queue;  // the dispatcher waits for requests
  std::deque<hg_ticket*> queue;
  bool stop = false;
  uint64_t batches = 0, requests = 0;
  std::thread th;
  // dispatcher-owned staging of one batch
  std::vector<hg_request> reqs;
  std::vector<uint64_t> words;
  std::vector<uint8_t> sigs;
  std::vector<int32_t> codes;
  void run();
};

void hg_batcher::run() {
  std::unique_lock<std::mutex> lk(mu);
  for (;;) {
    cv_queue.wait(lk, [&] { return stop || !queue.empty(); });
    if (queue.empty()) return;  // stop requested and drained
    // linger for more requests, bounded by the oldest request's wait: requests
    // that queued up while the previous batch ran go out at once
    const auto deadline = queue.front()->t_submit + max_wait;
    while (!stop && queue.size() < max_batch && std::chrono::steady_clock::now() < deadline)
      cv_queue.wait_until(lk, deadline);
    // one batch: the oldest request's message, up to max_batch requests of it
    std::vector<hg_ticket*> take;
    const std::string msg = queue.front()->msg;
    for (auto it = queue.begin(); it != queue.end() && take.size() < max_batch;) {
      if ((*it)->msg == msg) {
        take.push_back(*it);
        it = queue.erase(it);
      } else {
        ++it;
      }
    }
    lk.unlock();
    const size_t n = take.size();
    reqs.resize(n);
    sigs.resize(64 * n);
    codes.assign(n, HG_OK);
    words.clear();
    for (size_t i = 0; i < n; i++) {
      hg_request r = take[i]->req;
      r.word_offset = (uint32_t)words.size();
      reqs[i] = r;
      words.insert(words.end(), take[i]->words.begin(), take[i]->words.end());
      memcpy(&sigs[64 * i], take[i]->sig, 64);
    }
    const int rc = hg_verify_aggregate_msg(ctx, reinterpret_cast<const uint8_t*>(msg.data()), msg.size(),
                                           reqs.data(), n, words.empty() ? nullptr : words.data(), words.size(),
                                           sigs.data(), codes.data(), nullptr);
    // notify under each ticket's lock: once it is released the waiter may
    // delete the ticket, so nothing touches it afterwards
    for (size_t i = 0; i < n; i++) {
      hg_ticket* t = take[i];
      std::lock_guard<std::mutex> g(t->mu);
      t->rc = rc;
      t->code = rc == HG_OK ? codes[i] : rc;
      t->done = true;
      t->cv.notify_one();
    }
    lk.lock();
    batches++;
    requests += n;
  }
}

extern "C" {

int hg_batcher_create(hg_ctx* ctx, size_t max_batch, unsigned max_wait_us, hg_batcher** out) {
  if (!ctx || !out || max_batch == 0 || max_batch > (size_t)INT32_MAX) return HG_ERR_ARG;
  hg_batcher* b = new hg_batcher();
  b->ctx = ctx;
  b->max_batch = max_batch;
  b->max_wait = std::chrono::microseconds(max_wait_us);
  b->th = std::thread([b] { b->run(); });
  *out = b;
  return HG_OK;
}

void hg_batcher_destroy(hg_batcher* b) {
  if (!b) return;
  {
    std::lock_guard<std::mutex> g(b->mu);
    b->stop = true;
  }
  b->cv_queue.notify_all();
  b->th.join();  // queued requests are verified first; their callers still own the tickets
  delete b;       // tickets never point back at the batcher
}

int hg_batcher_submit(hg_batcher* b, const uint8_t* msg, size_t len, const hg_request* req, const uint64_t* words,
                      const uint8_t* sig, hg_ticket** out) {
  if (!b || !req || !sig || !out || (!msg && len)) return HG_ERR_ARG;
  const size_t nw = ((size_t)req->bitlen + 63) / 64;
  if (nw && !words) return HG_ERR_ARG;
  hg_ticket* t = new hg_ticket();
  t->msg.assign(reinterpret_cast<const char*>(msg), len);
  t->req = *req;
  t->words.assign(words, words + nw);
  memcpy(t->sig, sig, 64);
  t->t_submit = std::chrono::steady_clock::now();
  {
    std::lock_guard<std::mutex> g(b->mu);
    if (b->stop) {
      delete t;
      return HG_ERR_ARG;
    }
    b->queue.push_back(t);
  }
  b->cv_queue.notify_one();
  *out = t;
  return HG_OK;
}

int hg_batcher_wait(hg_batcher* b, hg_ticket* t, int32_t* code) {
  (void)b;  // the ticket holds everything (it may outlive the batcher)
  if (!t) return HG_ERR_ARG;
  int rc;
  {
    std::unique_lock<std::mutex> lk(t->mu);
    t->cv.wait(lk, [&] { return t->done; });
    rc = t->rc;
    if (code) *code = t->code;
  }
  delete t;
  return rc;
}

int hg_batcher_verify_aggregate(hg_batcher* b, const uint8_t* msg, size_t len, const hg_request* req,
                                const uint64_t* words, const uint8_t* sig, int32_t* code) {
  hg_ticket* t = nullptr;
  int rc = hg_batcher_submit(b, msg, len, req, words, sig, &t);
  if (rc) return rc;
  return hg_batcher_wait(b, t, code);
}

int hg_batcher_stats(hg_batcher* b, uint64_t* batches, uint64_t* requests) {
  if (!b) return HG_ERR_ARG;
  std::lock_guard<std::mutex> g(b->mu);
  if (batches) *batches = b->batches;
  if (requests) *requests = b->requests;
  return HG_OK;
}

}  // extern "C"
