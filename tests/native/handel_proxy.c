/*
 * handel_proxy.c — a process-model proxy of BASELINE config 4 (simul's
 * 2000-node single-host run with every evaluator check offloaded to one GPU).
 * NOT Handel completion time: it reproduces the verification load and the
 * process layout, not the protocol.
 *
 * Layout (simul/node/main.go:33-144): P OS processes, each running K Handel
 * instances (nodes p*K .. p*K+K-1 of an N-node registry). Every instance's
 * processLoop checks one incoming multisignature at a time
 * (processing.go:228-287 -> verifySignature :342-368); here an instance issues
 * R checks one after another, each a random level of its node (partitioner.go
 * rangeLevel :133-178), a bitset of density U[0.5, 1], the aggregate
 * signature of the set bits (every 8th tampered). Each process owns one
 * verification context (its own registry copy and GT tables in HBM) and one
 * hg_batcher that merges its instances' concurrent checks into GPU batches.
 * W worker threads per process drive the K instances (an instance has at most
 * one check in flight, like a processLoop); per-check latency is measured
 * from submission to verdict.
 *
 * The parent never loads the HIP library: each child is forked first and then
 * dlopen()s it, so no process ever forks with an initialised GPU runtime.
 *
 * Usage: handel_proxy <libhandel_gpu.so> [options]
 *   -p P   processes (8)        -k K  instances per process (250)
 *   -n N   registry keys (2000) -r R  checks per instance (45)
 *   -w W   worker threads per process (16)
 *   -b B   batcher max batch (4096)  -u U  batcher max wait, us (200)
 *   -P 0|1 hg_prepare_aggregate before the run (0: the volume policy)
 *   -L l   pin the table level (-1: policy, default)
 *   -M MB  GT table budget per process (default unlimited)
 *   -d DIR process 0 writes reg.bin, reqs.bin, words.bin, sigs.bin,
 *          codes.bin (its requests and the GPU's verdicts) for an oracle check
 * Prints one JSON line; exit 0 iff every verdict is the expected one.
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <errno.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

#include "handel_gpu.h"

static const uint8_t kMsg[] = "Everything that is beautiful and noble is the product of reason and calculation.";
#define MSG_LEN (sizeof kMsg - 1) /* lib.Message, simul/lib/config.go:37 */

/* ---------------------------------------------------------------- the C ABI, resolved after fork */
static struct {
  int (*create)(int, int, hg_ctx**);
  void (*destroy)(hg_ctx*);
  const char* (*last_error)(hg_ctx*);
  int (*registry_load)(hg_ctx*, const uint8_t*, size_t, int32_t*);
  int (*set_message)(hg_ctx*, const uint8_t*, size_t);
  int (*keygen)(hg_ctx*, const uint8_t*, size_t, uint8_t*);
  int (*sign)(hg_ctx*, const uint8_t*, size_t, uint8_t*);
  int (*prepare)(hg_ctx*);
  int (*tables)(hg_ctx*);
  int (*set_level)(hg_ctx*, int);
  int (*set_budget)(hg_ctx*, size_t);
  size_t (*ctx_bytes)(hg_ctx*);
  int (*b_create)(hg_ctx*, size_t, unsigned, hg_batcher**);
  void (*b_destroy)(hg_batcher*);
  int (*b_submit)(hg_batcher*, const uint8_t*, size_t, const hg_request*, const uint64_t*, const uint8_t*,
                  hg_ticket**);
  int (*b_wait)(hg_batcher*, hg_ticket*, int32_t*);
  int (*b_stats)(hg_batcher*, uint64_t*, uint64_t*);
} A;

static void resolve(const char* path) {
  void* h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
  if (!h) {
    fprintf(stderr, "dlopen %s: %s\n", path, dlerror());
    exit(3);
  }
#define R_(field, name)                                    \
  do {                                                     \
    *(void**)(&A.field) = dlsym(h, name);                  \
    if (!A.field) {                                        \
      fprintf(stderr, "missing symbol %s\n", name);        \
      exit(3);                                             \
    }                                                      \
  } while (0)
  R_(create, "hg_create");
  R_(destroy, "hg_destroy");
  R_(last_error, "hg_last_error");
  R_(registry_load, "hg_registry_load");
  R_(set_message, "hg_set_message");
  R_(keygen, "hg_keygen");
  R_(sign, "hg_sign");
  R_(prepare, "hg_prepare_aggregate");
  R_(tables, "hg_aggregate_tables");
  R_(set_level, "hg_set_aggregate_level");
  R_(set_budget, "hg_set_table_budget");
  R_(ctx_bytes, "hg_context_bytes");
  R_(b_create, "hg_batcher_create");
  R_(b_destroy, "hg_batcher_destroy");
  R_(b_submit, "hg_batcher_submit");
  R_(b_wait, "hg_batcher_wait");
  R_(b_stats, "hg_batcher_stats");
#undef R_
}

/* ---------------------------------------------------------------- helpers */
static double now_s(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

static uint64_t splitmix(uint64_t* s) {
  uint64_t z = (*s += 0x9e3779b97f4a7c15ull);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
static double unif(uint64_t* s) { return (double)(splitmix(s) >> 11) * (1.0 / 9007199254740992.0); }

/* the group order n, little-endian 64-bit limbs */
static const uint64_t kN[4] = {0x1a2ef45b57ac7261ull, 0x2e8d8e12f82b3924ull, 0xaa6fecb86184dc21ull,
                               0x8fb501e34aa387f9ull};
static int geq_n(const uint64_t a[4]) {
  for (int i = 3; i >= 0; i--) {
    if (a[i] != kN[i]) return a[i] > kN[i];
  }
  return 1;
}
/* a = (a + b) mod n, a, b < n */
static void add_mod_n(uint64_t a[4], const uint64_t b[4]) {
  unsigned __int128 c = 0;
  uint64_t r[4];
  for (int i = 0; i < 4; i++) {
    c += (unsigned __int128)a[i] + b[i];
    r[i] = (uint64_t)c;
    c >>= 64;
  }
  if (c || geq_n(r)) {
    unsigned __int128 br = 0;
    for (int i = 0; i < 4; i++) {
      unsigned __int128 d = (unsigned __int128)r[i] - kN[i] - (uint64_t)br;
      r[i] = (uint64_t)d;
      br = (d >> 64) ? 1 : 0;
    }
  }
  memcpy(a, r, sizeof r);
}
static void to_be(uint8_t out[32], const uint64_t a[4]) {
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 8; j++) out[31 - 8 * i - j] = (uint8_t)(a[i] >> (8 * j));
}

/* binomialPartitioner.rangeLevel (partitioner.go:133-178); 0 if the level is empty */
static int range_level(uint32_t id, uint32_t size, int level, uint32_t* lo, uint32_t* hi) {
  int bitsize = 0;
  while ((1u << bitsize) < size) bitsize++;
  uint32_t a = 0, b = 1u << bitsize;
  int inverse = level - 1, idx = bitsize - 1;
  while (idx >= inverse && idx >= 0 && a < b) {
    uint32_t mid = (a + b) / 2;
    int bit = (id >> idx) & 1;
    if ((bit == 1) == (idx == inverse)) b = mid;
    else a = mid;
    idx--;
  }
  if (a >= size) return 0;
  *lo = a;
  *hi = b < size ? b : size;
  return 1;
}

/* ---------------------------------------------------------------- one process */
typedef struct {
  int procs, inst, nreg, checks, workers, max_batch, wait_us, prepare, level;
  long budget_mb;
  const char* dump;
  const char* lib;
} opts;

typedef struct {
  double t0, t1, setup_s, prepare_s;
  uint64_t requests, batches, mismatches, ctx_bytes;
  int tables_before, tables_after, rc;
} proc_result;

typedef struct {
  hg_request req;
  uint32_t word_off, nw;
  int32_t expect, got;
} check;

static hg_batcher* g_b;
static check* g_checks;
static uint64_t* g_words;
static uint8_t* g_sigs;
static double* g_lat;
static const opts* g_o;
static int g_fail;

typedef struct {
  int w;
} worker_arg;

static void* worker(void* arg) {
  const int w = ((worker_arg*)arg)->w;
  const opts* o = g_o;
  /* instances w, w + W, w + 2W, ... of this process; one check each in flight */
  int mine = 0;
  for (int i = w; i < o->inst; i += o->workers) mine++;
  hg_ticket** t = (hg_ticket**)calloc((size_t)mine, sizeof(hg_ticket*));
  double* ts = (double*)calloc((size_t)mine, sizeof(double));
  for (int step = 0; step < o->checks; step++) {
    int j = 0;
    for (int i = w; i < o->inst; i += o->workers, j++) {
      check* c = &g_checks[(size_t)i * o->checks + step];
      ts[j] = now_s();
      if (A.b_submit(g_b, kMsg, MSG_LEN, &c->req, g_words + c->word_off, g_sigs + 64 * ((size_t)i * o->checks + step),
                     &t[j]) != HG_OK)
        g_fail = 1;
    }
    j = 0;
    for (int i = w; i < o->inst; i += o->workers, j++) {
      const size_t k = (size_t)i * o->checks + step;
      int32_t code = -1;
      if (A.b_wait(g_b, t[j], &code) != HG_OK) g_fail = 1;
      g_lat[k] = now_s() - ts[j];
      g_checks[k].got = code;
    }
  }
  free(t);
  free(ts);
  return NULL;
}

static int write_file(const char* dir, const char* name, const void* p, size_t n) {
  char path[4096];
  snprintf(path, sizeof path, "%s/%s", dir, name);
  FILE* f = fopen(path, "wb");
  if (!f) return -1;
  size_t k = n ? fwrite(p, 1, n, f) : 0;
  fclose(f);
  return k == n ? 0 : -1;
}

static int cmp_double(const void* a, const void* b) {
  double x = *(const double*)a, y = *(const double*)b;
  return (x > y) - (x < y);
}

static void run_process(const opts* o, int p, int ready_fd, int start_fd, int out_fd) {
  proc_result res;
  memset(&res, 0, sizeof res);
  g_o = o;
  resolve(o->lib);
  const double ts0 = now_s();
  hg_ctx* ctx = NULL;
  if (A.create(0, HG_FLAVOR_GO, &ctx) != HG_OK) {
    fprintf(stderr, "proc %d: hg_create failed\n", p);
    exit(4);
  }
  if (o->level != -1) A.set_level(ctx, o->level);
  if (o->budget_mb >= 0) A.set_budget(ctx, (size_t)o->budget_mb << 20);
  /* the registry: the same seeded keys in every process (simul's shared registry file) */
  const size_t N = (size_t)o->nreg;
  uint64_t* sk = (uint64_t*)malloc(N * 4 * sizeof(uint64_t));
  uint8_t* skb = (uint8_t*)malloc(N * 32);
  uint64_t seed = 0x48616e64656cull;
  for (size_t i = 0; i < N; i++) {
    for (int j = 0; j < 4; j++) sk[4 * i + j] = splitmix(&seed);
    sk[4 * i + 3] &= 0x0fffffffffffffffull; /* < n */
    sk[4 * i] |= 1;                         /* > 0 */
    to_be(skb + 32 * i, sk + 4 * i);
  }
  uint8_t* reg = (uint8_t*)malloc(N * 128);
  int rc = A.set_message(ctx, kMsg, MSG_LEN);
  if (rc == HG_OK) rc = A.keygen(ctx, skb, N, reg);
  if (rc == HG_OK) rc = A.registry_load(ctx, reg, N, NULL);
  if (rc != HG_OK) {
    fprintf(stderr, "proc %d: setup rc %d: %s\n", p, rc, A.last_error(ctx));
    exit(4);
  }
  /* this process's checks: K instances x R */
  const size_t nchk = (size_t)o->inst * o->checks;
  g_checks = (check*)calloc(nchk, sizeof(check));
  size_t cap_words = nchk * ((N + 63) / 64 + 1);
  g_words = (uint64_t*)calloc(cap_words, sizeof(uint64_t));
  uint8_t* agg_sk = (uint8_t*)malloc(nchk * 32);
  g_sigs = (uint8_t*)malloc(nchk * 64);
  g_lat = (double*)calloc(nchk, sizeof(double));
  uint64_t rs = 0x5eedull + (uint64_t)p * 7919u;
  size_t wpos = 0;
  for (int i = 0; i < o->inst; i++) {
    const uint32_t node = (uint32_t)((p * o->inst + i) % o->nreg);
    uint32_t lo[32], hi[32];
    int nl = 0;
    for (int lvl = 1; lvl <= 31 && (1u << (lvl - 1)) < (uint32_t)o->nreg; lvl++)
      if (range_level(node, (uint32_t)o->nreg, lvl, &lo[nl], &hi[nl])) nl++;
    for (int s = 0; s < o->checks; s++) {
      const size_t k = (size_t)i * o->checks + s;
      check* c = &g_checks[k];
      const int l = (int)(splitmix(&rs) % (uint64_t)nl);
      const uint32_t size = hi[l] - lo[l];
      const double dens = 0.5 + 0.5 * unif(&rs);
      c->req.offset = lo[l];
      c->req.bitlen = size;
      c->req.level_size = size;
      c->word_off = (uint32_t)wpos;
      c->nw = (size + 63) / 64;
      c->req.word_offset = (uint32_t)wpos;
      uint64_t acc[4] = {0, 0, 0, 0};
      const uint32_t forced = (uint32_t)(splitmix(&rs) % size);
      for (uint32_t b = 0; b < size; b++) {
        if (b == forced || unif(&rs) < dens) {
          g_words[wpos + b / 64] |= 1ull << (b % 64);
          add_mod_n(acc, sk + 4 * (lo[l] + b));
        }
      }
      wpos += c->nw;
      c->expect = HG_OK;
      if (k % 8 == 0) { /* tamper: sign k + 1 */
        const uint64_t one[4] = {1, 0, 0, 0};
        add_mod_n(acc, one);
        c->expect = HG_ERR_SIG_INVALID;
      }
      to_be(agg_sk + 32 * k, acc);
    }
  }
  rc = A.sign(ctx, agg_sk, nchk, g_sigs);
  if (rc != HG_OK) {
    fprintf(stderr, "proc %d: sign rc %d: %s\n", p, rc, A.last_error(ctx));
    exit(4);
  }
  res.setup_s = now_s() - ts0;
  res.tables_before = A.tables(ctx);
  if (o->prepare) {
    const double tp = now_s();
    if (A.prepare(ctx) != HG_OK) {
      fprintf(stderr, "proc %d: prepare: %s\n", p, A.last_error(ctx));
      exit(4);
    }
    res.prepare_s = now_s() - tp;
  }
  if (A.b_create(ctx, (size_t)o->max_batch, (unsigned)o->wait_us, &g_b) != HG_OK) exit(4);
  /* ready, then wait for the common start */
  char c1 = 'r';
  if (write(ready_fd, &c1, 1) != 1) exit(5);
  if (read(start_fd, &c1, 1) != 1) exit(5);
  pthread_t th[256];
  worker_arg wa[256];
  res.t0 = now_s();
  for (int w = 0; w < o->workers; w++) {
    wa[w].w = w;
    pthread_create(&th[w], NULL, worker, &wa[w]);
  }
  for (int w = 0; w < o->workers; w++) pthread_join(th[w], NULL);
  res.t1 = now_s();
  A.b_stats(g_b, &res.batches, &res.requests);
  A.b_destroy(g_b);
  res.tables_after = A.tables(ctx);
  res.ctx_bytes = A.ctx_bytes(ctx);
  for (size_t k = 0; k < nchk; k++) res.mismatches += g_checks[k].got != g_checks[k].expect;
  res.rc = g_fail;
  if (o->dump && p == 0) {
    hg_request* rq = (hg_request*)malloc(nchk * sizeof(hg_request));
    int32_t* got = (int32_t*)malloc(nchk * sizeof(int32_t));
    for (size_t k = 0; k < nchk; k++) {
      rq[k] = g_checks[k].req;
      got[k] = g_checks[k].got;
    }
    if (write_file(o->dump, "reg.bin", reg, N * 128) || write_file(o->dump, "reqs.bin", rq, nchk * sizeof(hg_request)) ||
        write_file(o->dump, "words.bin", g_words, wpos * 8) || write_file(o->dump, "sigs.bin", g_sigs, nchk * 64) ||
        write_file(o->dump, "codes.bin", got, nchk * 4))
      res.rc = 1;
    free(rq);
    free(got);
  }
  A.destroy(ctx);
  /* result, then the latencies */
  if (write(out_fd, &res, sizeof res) != (ssize_t)sizeof res) exit(5);
  size_t off = 0, bytes = nchk * sizeof(double);
  while (off < bytes) {
    ssize_t k = write(out_fd, (const char*)g_lat + off, bytes - off);
    if (k <= 0) exit(5);
    off += (size_t)k;
  }
  exit(0);
}

static int read_full(int fd, void* p, size_t n) {
  size_t off = 0;
  while (off < n) {
    ssize_t k = read(fd, (char*)p + off, n - off);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) return -1;
    off += (size_t)k;
  }
  return 0;
}

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: %s <libhandel_gpu.so> [-p P] [-k K] [-n N] [-r R] [-w W] [-b B] [-u U] [-P 0|1] "
                    "[-L level] [-M MB] [-d DIR]\n", argv[0]);
    return 2;
  }
  opts o = {8, 250, 2000, 45, 16, 4096, 200, 0, -1, -1, NULL, argv[1]};
  for (int i = 2; i + 1 < argc; i += 2) {
    const char* f = argv[i];
    const char* v = argv[i + 1];
    if (!strcmp(f, "-p")) o.procs = atoi(v);
    else if (!strcmp(f, "-k")) o.inst = atoi(v);
    else if (!strcmp(f, "-n")) o.nreg = atoi(v);
    else if (!strcmp(f, "-r")) o.checks = atoi(v);
    else if (!strcmp(f, "-w")) o.workers = atoi(v);
    else if (!strcmp(f, "-b")) o.max_batch = atoi(v);
    else if (!strcmp(f, "-u")) o.wait_us = atoi(v);
    else if (!strcmp(f, "-P")) o.prepare = atoi(v);
    else if (!strcmp(f, "-L")) o.level = atoi(v);
    else if (!strcmp(f, "-M")) o.budget_mb = atol(v);
    else if (!strcmp(f, "-d")) o.dump = v;
    else {
      fprintf(stderr, "unknown option %s\n", f);
      return 2;
    }
  }
  if (o.procs < 1 || o.procs > 15 || o.inst < 1 || o.nreg < 2 || o.checks < 1 || o.workers < 1 ||
      o.workers > 256 || o.workers > o.inst || o.max_batch < 1) {
    fprintf(stderr, "bad options (1 <= procs <= 15, 1 <= workers <= min(256, instances))\n");
    return 2;
  }
  pid_t pid[16];
  int ready[16][2], start[16][2], out[16][2];
  for (int p = 0; p < o.procs; p++) {
    if (pipe(ready[p]) || pipe(start[p]) || pipe(out[p])) return 6;
    pid[p] = fork();
    if (pid[p] < 0) return 6;
    if (pid[p] == 0) {
      close(ready[p][0]);
      close(start[p][1]);
      close(out[p][0]);
      run_process(&o, p, ready[p][1], start[p][0], out[p][1]);
    }
    close(ready[p][1]);
    close(start[p][0]);
    close(out[p][1]);
  }
  int bad = 0;
  for (int p = 0; p < o.procs; p++) {
    char c;
    if (read_full(ready[p][0], &c, 1)) bad = 1;
  }
  for (int p = 0; p < o.procs; p++) {
    char c = 's';
    if (write(start[p][1], &c, 1) != 1) bad = 1;
  }
  const size_t nchk = (size_t)o.inst * o.checks;
  double* lat = (double*)malloc(nchk * o.procs * sizeof(double));
  proc_result r[16];
  for (int p = 0; p < o.procs; p++) {
    if (read_full(out[p][0], &r[p], sizeof r[p]) || read_full(out[p][0], lat + nchk * p, nchk * sizeof(double))) {
      fprintf(stderr, "process %d: no result\n", p);
      bad = 1;
      memset(&r[p], 0, sizeof r[p]);
    }
  }
  for (int p = 0; p < o.procs; p++) {
    int st = 0;
    waitpid(pid[p], &st, 0);
    if (!WIFEXITED(st) || WEXITSTATUS(st) != 0) bad = 1;
  }
  if (bad) {
    fprintf(stderr, "handel_proxy: a process failed\n");
    return 1;
  }
  double t0 = r[0].t0, t1 = r[0].t1, setup = 0, prep = 0;
  uint64_t reqs = 0, batches = 0, mism = 0, bytes_max = 0;
  int fails = 0, tb = r[0].tables_before, ta = r[0].tables_after;
  for (int p = 0; p < o.procs; p++) {
    if (r[p].t0 < t0) t0 = r[p].t0;
    if (r[p].t1 > t1) t1 = r[p].t1;
    if (r[p].setup_s > setup) setup = r[p].setup_s;
    if (r[p].prepare_s > prep) prep = r[p].prepare_s;
    if (r[p].ctx_bytes > bytes_max) bytes_max = r[p].ctx_bytes;
    reqs += r[p].requests;
    batches += r[p].batches;
    mism += r[p].mismatches;
    fails += r[p].rc;
  }
  qsort(lat, nchk * o.procs, sizeof(double), cmp_double);
  const size_t m = nchk * o.procs;
  const double wall = t1 - t0;
  printf("{\"harness\": \"handel_proxy\", \"what\": \"config-4 process-model proxy (not Handel completion time)\", "
         "\"procs\": %d, \"instances_per_proc\": %d, \"nodes\": %d, \"registry\": %d, \"checks_per_instance\": %d, "
         "\"workers_per_proc\": %d, \"prepare\": %d, \"tables_before\": %d, \"tables_after\": %d, "
         "\"requests\": %llu, \"batches\": %llu, \"mean_batch\": %.1f, \"wall_ms\": %.3f, "
         "\"throughput\": %.1f, \"latency_us\": {\"p50\": %.1f, \"p90\": %.1f, \"p99\": %.1f, \"max\": %.1f}, "
         "\"hbm_per_proc_bytes\": %llu, \"setup_s_max\": %.3f, \"prepare_ms_max\": %.3f, \"mismatches\": %llu}\n",
         o.procs, o.inst, o.procs * o.inst, o.nreg, o.checks, o.workers, o.prepare, tb, ta,
         (unsigned long long)reqs, (unsigned long long)batches, batches ? (double)reqs / batches : 0.0, wall * 1e3,
         wall > 0 ? reqs / wall : 0.0, 1e6 * lat[m / 2], 1e6 * lat[(m * 9) / 10], 1e6 * lat[(m * 99) / 100],
         1e6 * lat[m - 1], (unsigned long long)bytes_max, setup, prep * 1e3, (unsigned long long)mism);
  free(lat);
  return (mism || fails || reqs != m) ? 1 : 0;
}
