/*
 * abi_threads.c — C-level test of the C ABI's thread-safety contract
 * (include/handel_gpu.h: "every entry point is thread-safe per context"),
 * the way a cgo caller uses it: k Handel instances in one process
 * (simul/node/main.go:63-131) submitting to ONE shared context at once.
 *
 * Test infrastructure, built by handel_amd/build.py (gcc, links only the
 * C ABI) and run as a fresh process by tests/test_gpu_boundary.py, which
 * writes the fixtures and their expected results (checked against the
 * oracle there) into a directory:
 *   reg.bin   registry marshals (n_reg x 128)
 *   reqs.bin  hg_request x n_req     words.bin  uint64 bitset words
 *   asigs.bin aggregate sigs on message 1 (n_req x 64)  acodes.bin expected codes
 *   agg.bin   expected aggregate-key marshals (n_req x 128)
 *   msgK.bin, pksK.bin, sigsK.bin, codesK.bin (K = 1, 2): single checks on
 *             two DIFFERENT messages
 *
 * Usage: abi_threads <fixture dir> <threads> <iterations>
 * Threads alternate between aggregate batches on message 1
 * (hg_verify_aggregate_msg) and single-check batches on message 1 or 2
 * (hg_verify_batch_msg), so the context's cached hashed message flips
 * between calls while other threads' batches are in flight. Every result is compared with the
 * expected bytes; prints "abi_threads ok <calls>" and exits 0 on success.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "handel_gpu.h"

typedef struct {
  uint8_t* p;
  size_t n;
} blob;

static blob load(const char* dir, const char* name) {
  char path[4096];
  snprintf(path, sizeof path, "%s/%s", dir, name);
  FILE* f = fopen(path, "rb");
  blob b = {0, 0};
  if (!f) {
    fprintf(stderr, "cannot open %s\n", path);
    exit(2);
  }
  fseek(f, 0, SEEK_END);
  b.n = (size_t)ftell(f);
  fseek(f, 0, SEEK_SET);
  b.p = (uint8_t*)malloc(b.n ? b.n : 1);
  if (b.n && fread(b.p, 1, b.n, f) != b.n) {
    fprintf(stderr, "short read %s\n", path);
    exit(2);
  }
  fclose(f);
  return b;
}

static hg_ctx* ctx;
static blob reqs, words, asigs, acodes, agg;
static blob msg[2], pks[2], sigs[2], codes[2];
static int iters;
static int failures;
static long calls;
static pthread_mutex_t mu = PTHREAD_MUTEX_INITIALIZER;

static void fail(int tid, const char* what, int it) {
  pthread_mutex_lock(&mu);
  failures++;
  fprintf(stderr, "thread %d iteration %d: %s (%s)\n", tid, it, what, hg_last_error(ctx));
  pthread_mutex_unlock(&mu);
}

static void* worker(void* arg) {
  int tid = (int)(intptr_t)arg;
  size_t nreq = reqs.n / sizeof(hg_request);
  int32_t* got = (int32_t*)malloc(sizeof(int32_t) * (nreq + pks[0].n / 128 + pks[1].n / 128 + 1));
  uint8_t* got_agg = (uint8_t*)malloc(nreq * 128 + 1);
  for (int it = 0; it < iters; it++) {
    int kind = (tid + it) % 3;  /* 0: aggregate, 1: message 1, 2: message 2 */
    if (kind == 0) {
      int rc = hg_verify_aggregate_msg(ctx, msg[0].p, msg[0].n, (const hg_request*)reqs.p, nreq,
                                       (const uint64_t*)words.p, words.n / 8, asigs.p, got, got_agg);
      if (rc != HG_OK) fail(tid, "hg_verify_aggregate_msg rc", it);
      else if (memcmp(got, acodes.p, acodes.n) != 0) fail(tid, "aggregate codes differ", it);
      else if (memcmp(got_agg, agg.p, agg.n) != 0) fail(tid, "aggregate keys differ", it);
    } else {
      int k = kind - 1;
      size_t n = sigs[k].n / 64;
      int rc = hg_verify_batch_msg(ctx, msg[k].p, msg[k].n, pks[k].p, sigs[k].p, n, got);
      if (rc != HG_OK) fail(tid, "hg_verify_batch_msg rc", it);
      else if (memcmp(got, codes[k].p, codes[k].n) != 0) fail(tid, "single-check codes differ", it);
    }
    pthread_mutex_lock(&mu);
    calls++;
    pthread_mutex_unlock(&mu);
  }
  free(got);
  free(got_agg);
  return NULL;
}

int main(int argc, char** argv) {
  if (argc != 4) {
    fprintf(stderr, "usage: %s <fixture dir> <threads> <iterations>\n", argv[0]);
    return 2;
  }
  const char* dir = argv[1];
  int nthreads = atoi(argv[2]);
  iters = atoi(argv[3]);
  if (nthreads < 1 || nthreads > 64 || iters < 1) return 2;
  blob reg = load(dir, "reg.bin");
  reqs = load(dir, "reqs.bin");
  words = load(dir, "words.bin");
  asigs = load(dir, "asigs.bin");
  acodes = load(dir, "acodes.bin");
  agg = load(dir, "agg.bin");
  for (int k = 0; k < 2; k++) {
    char name[64];
    snprintf(name, sizeof name, "msg%d.bin", k + 1);
    msg[k] = load(dir, name);
    snprintf(name, sizeof name, "pks%d.bin", k + 1);
    pks[k] = load(dir, name);
    snprintf(name, sizeof name, "sigs%d.bin", k + 1);
    sigs[k] = load(dir, name);
    snprintf(name, sizeof name, "codes%d.bin", k + 1);
    codes[k] = load(dir, name);
  }
  if (hg_create(0, HG_FLAVOR_GO, &ctx) != HG_OK) {
    fprintf(stderr, "hg_create failed\n");
    return 1;
  }
  int rc = hg_registry_load(ctx, reg.p, reg.n / 128, NULL);
  if (rc != HG_OK) {
    fprintf(stderr, "hg_registry_load: %d %s\n", rc, hg_last_error(ctx));
    return 1;
  }
  pthread_t th[64];
  for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, worker, (void*)(intptr_t)t);
  for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
  hg_destroy(ctx);
  if (failures) {
    fprintf(stderr, "abi_threads: %d failures in %ld calls\n", failures, calls);
    return 1;
  }
  printf("abi_threads ok %ld\n", calls);
  return 0;
}
