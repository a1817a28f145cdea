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
 * signature of the set bits (every 8th tampered). Per-check latency is
 * measured from submission to verdict. Two process models:
 *
 *   -D 0 (contexts): each process owns one verification context (its own
 *        registry copy and GT tables in HBM) and one hg_batcher that merges
 *        its instances' concurrent checks; W worker threads per process drive
 *        the K instances (an instance has at most one check in flight).
 *   -D 1 (daemon): ONE server process owns the GPU context, the registry and
 *        one set of GT tables and runs the verifier service (hg_service_*);
 *        the P client processes load only libhandel_client.so (no GPU) and
 *        submit through the shared-memory region. Each client process runs W
 *        poller threads (default 1), each one handle driving its share of the
 *        K instances as an event loop (wait_any, then the instance's next check).
 *
 * The parent never loads the HIP library: every child is forked first and
 * then dlopen()s what it needs, so no process forks with an initialised GPU
 * runtime. The workload lives in one anonymous shared mapping made by the
 * parent: process p's checks are generated (and, in daemon mode, signed by
 * the server) there, and the verdicts land there for the parent to check.
 *
 * Usage: handel_proxy <libhandel_gpu.so> [options]
 *   -p P   processes (8)        -k K  instances per process (250)
 *   -n N   registry keys (2000) -r R  checks per instance (45)
 *   -w W   worker threads per process (16; daemon mode: poller threads, 4)
 *   -b B   max batch (4096)     -u U  max wait, us (200; daemon mode 50)
 *   -P 0|1 prepare the GT tables before the run (0: the volume policy)
 *   -L l   pin the table level (-1: policy, default)
 *   -M MB  GT table budget per context (default unlimited)
 *   -D 0|1 process model (0: a context per process, 1: the verifier service)
 *   -l L   daemon: lanes (batches in flight, 8)   -o 0|1 daemon: fold overlap (1)
 *   -Q q   daemon: GPU_MAX_HW_QUEUES of the server (default 2 x lanes: a lane's two streams
 *          each on a hardware queue of their own)
 *   -q us  daemon: launch once no request has arrived for us microseconds (0: off)
 *   -F 0|1 daemon: launch once every request the finished batches released is back (1)
 *   -E us  daemon: serve with the CPU echo stand-in (no GPU; protocol test),
 *          each batch taking `us` microseconds
 *   -C lib daemon: libhandel_client.so (default: next to libhandel_gpu.so)
 *   -d DIR process 0's requests and verdicts for an oracle check: reg.bin,
 *          reqs.bin, words.bin, sigs.bin, codes.bin
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
#include <sys/mman.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

#include "handel_client.h"
#include "handel_gpu.h"

static const uint8_t kMsg[] = "Everything that is beautiful and noble is the product of reason and calculation.";
#define MSG_LEN (sizeof kMsg - 1) /* lib.Message, simul/lib/config.go:37 */

/* A forked child ends with _exit after flushing stdio: its atexit handlers
 * and static destructors are the PARENT's registrations, copied by fork. A
 * profiler's tool library preloaded into the parent (rocprofv3) registers its
 * finalizer there; run in two or more children at once it aborts inside
 * __cxa_finalize and its signal handler then never returns, so the parent's
 * waitpid hung (the contexts model under rocprofv3, diagnosed
 * from this proxy's stage log, tools/proxy_prof.py). The children release
 * their GPU contexts explicitly before this (hg_destroy); the kernel driver
 * reclaims the rest of a process at exit, as for any process. */
static void child_exit(int code) {
  fflush(NULL);
  _exit(code);
}

/* ---------------------------------------------------------------- the C ABIs, resolved after fork */
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
  void (*s_config_init)(hg_service_config*);
  int (*s_create)(hg_ctx*, const char*, const hg_service_config*, hg_service**);
  int (*s_create_echo)(const char*, const hg_service_config*, uint32_t, uint32_t, hg_service**);
  void (*s_destroy)(hg_service*);
  int (*s_stats)(hg_service*, uint64_t*, uint64_t*, uint64_t*);
} A;

static struct {
  int (*open)(const char*, hg_client**);
  void (*close)(hg_client*);
  int (*submit)(hg_client*, const uint8_t*, size_t, const hg_request*, const uint64_t*, const uint8_t*, uint64_t*);
  int (*wait_any)(hg_client*, uint64_t*, int32_t*, size_t, long);
} C;

static void* open_lib(const char* path) {
  void* h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
  if (!h) {
    fprintf(stderr, "dlopen %s: %s\n", path, dlerror());
    child_exit(3);
  }
  return h;
}
#define R_(S, h, field, name)                              \
  do {                                                     \
    *(void**)(&S.field) = dlsym(h, name);                  \
    if (!S.field) {                                        \
      fprintf(stderr, "missing symbol %s\n", name);        \
      child_exit(3);                                             \
    }                                                      \
  } while (0)

static void resolve_gpu(const char* path) {
  void* h = open_lib(path);
  R_(A, h, create, "hg_create");
  R_(A, h, destroy, "hg_destroy");
  R_(A, h, last_error, "hg_last_error");
  R_(A, h, registry_load, "hg_registry_load");
  R_(A, h, set_message, "hg_set_message");
  R_(A, h, keygen, "hg_keygen");
  R_(A, h, sign, "hg_sign");
  R_(A, h, prepare, "hg_prepare_aggregate");
  R_(A, h, tables, "hg_aggregate_tables");
  R_(A, h, set_level, "hg_set_aggregate_level");
  R_(A, h, set_budget, "hg_set_table_budget");
  R_(A, h, ctx_bytes, "hg_context_bytes");
  R_(A, h, b_create, "hg_batcher_create");
  R_(A, h, b_destroy, "hg_batcher_destroy");
  R_(A, h, b_submit, "hg_batcher_submit");
  R_(A, h, b_wait, "hg_batcher_wait");
  R_(A, h, b_stats, "hg_batcher_stats");
  R_(A, h, s_config_init, "hg_service_config_init");
  R_(A, h, s_create, "hg_service_create");
  R_(A, h, s_create_echo, "hg_service_create_echo");
  R_(A, h, s_destroy, "hg_service_destroy");
  R_(A, h, s_stats, "hg_service_stats");
}

static void resolve_client(const char* path) {
  void* h = open_lib(path);
  R_(C, h, open, "hg_client_open");
  R_(C, h, close, "hg_client_close");
  R_(C, h, submit, "hg_client_submit");
  R_(C, h, wait_any, "hg_client_wait_any");
}

/* ---------------------------------------------------------------- helpers */
static double now_s(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

/* one progress line per process phase on stderr (bench.py keeps the tail of
 * a run that times out, so a stall names the phase it stalled in) */
static double g_t_start;
static void stage(const char* who, int p, const char* what) {
  fprintf(stderr, "[proxy %.3f s] %s %d (pid %d): %s\n", now_s() - g_t_start, who, p, (int)getpid(), what);
  fflush(stderr);
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

/* ---------------------------------------------------------------- options and the shared workload */
typedef struct {
  int procs, inst, nreg, checks, workers, max_batch, wait_us, prepare, level, daemon, lanes, overlap, queues, quiet_us;
  long budget_mb, echo_us;
  int follow;
  const char* dump;
  const char* lib;
  const char* client_lib;
} opts;

typedef struct {
  hg_request req;
  uint32_t word_off, nw;
  int32_t expect, got;
} check;

/* per process p: checks[p], sigs[p], lat[p], words[p] (cap_words each) */
typedef struct {
  check* checks;
  uint8_t* sigs;
  uint8_t* agg_sk; /* the aggregate secret of each check (32 B big-endian), for signing */
  double* lat;
  uint64_t* words;
  size_t nchk, cap_words;
  size_t bytes;
} workload;

static workload W_;

static void workload_map(const opts* o) {
  const size_t nchk = (size_t)o->inst * o->checks, P = (size_t)o->procs;
  W_.nchk = nchk;
  W_.cap_words = nchk * (((size_t)o->nreg + 63) / 64 + 1);
  const size_t b_chk = P * nchk * sizeof(check), b_sig = P * nchk * 64, b_sk = P * nchk * 32,
               b_lat = P * nchk * sizeof(double), b_w = P * W_.cap_words * 8;
  W_.bytes = b_chk + b_sig + b_sk + b_lat + b_w;
  uint8_t* p = mmap(NULL, W_.bytes, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
  if (p == MAP_FAILED) {
    perror("mmap workload");
    exit(6);
  }
  W_.checks = (check*)p;
  W_.sigs = p + b_chk;
  W_.agg_sk = W_.sigs + b_sig;
  W_.lat = (double*)(W_.agg_sk + b_sk);
  W_.words = (uint64_t*)((uint8_t*)W_.lat + b_lat);
}

/* the registry's secret keys: the same seeded keys in every process (simul's shared registry file) */
static void registry_secrets(int nreg, uint64_t* sk, uint8_t* skb) {
  uint64_t seed = 0x48616e64656cull;
  for (int i = 0; i < nreg; i++) {
    for (int j = 0; j < 4; j++) sk[4 * i + j] = splitmix(&seed);
    sk[4 * i + 3] &= 0x0fffffffffffffffull; /* < n */
    sk[4 * i] |= 1;                         /* > 0 */
    to_be(skb + 32 * i, sk + 4 * i);
  }
}

/* process p's checks: requests, bitset words, expected codes, aggregate secrets.
 * echo: signatures for the CPU stand-in instead (sig[0] = tampered, sig[1..8] = xor of the words) */
static void gen_checks(const opts* o, int p, const uint64_t* sk, int echo) {
  const size_t nchk = W_.nchk;
  check* chk = W_.checks + (size_t)p * nchk;
  uint64_t* words = W_.words + (size_t)p * W_.cap_words;
  uint8_t* agg = W_.agg_sk + (size_t)p * nchk * 32;
  uint8_t* sigs = W_.sigs + (size_t)p * nchk * 64;
  memset(words, 0, W_.cap_words * 8);
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
      check* c = &chk[k];
      const int l = (int)(splitmix(&rs) % (uint64_t)nl);
      const uint32_t size = hi[l] - lo[l];
      const double dens = 0.5 + 0.5 * unif(&rs);
      c->req.offset = lo[l];
      c->req.bitlen = size;
      c->req.level_size = size;
      c->word_off = (uint32_t)wpos;
      c->nw = (size + 63) / 64;
      c->req.word_offset = (uint32_t)wpos;
      c->got = -1;
      uint64_t acc[4] = {0, 0, 0, 0};
      const uint32_t forced = (uint32_t)(splitmix(&rs) % size);
      for (uint32_t b = 0; b < size; b++) {
        if (b == forced || unif(&rs) < dens) {
          words[wpos + b / 64] |= 1ull << (b % 64);
          if (!echo) add_mod_n(acc, sk + 4 * (lo[l] + b));
        }
      }
      c->expect = HG_OK;
      if (k % 8 == 0) { /* tamper: sign k + 1 */
        const uint64_t one[4] = {1, 0, 0, 0};
        if (!echo) add_mod_n(acc, one);
        c->expect = HG_ERR_SIG_INVALID;
      }
      if (echo) {
        uint64_t x = 0;
        for (uint32_t j = 0; j < c->nw; j++) x ^= words[wpos + j];
        memset(sigs + 64 * k, 0, 64);
        sigs[64 * k] = c->expect == HG_OK ? 0 : 1;
        for (int b = 0; b < 8; b++) sigs[64 * k + 1 + b] = (uint8_t)(x >> (8 * b));
      } else {
        to_be(agg + 32 * k, acc);
      }
      wpos += c->nw;
    }
  }
}

typedef struct {
  double t0, t1, setup_s, prepare_s;
  uint64_t requests, batches, in_flight, ctx_bytes;
  int tables_before, tables_after, rc;
} proc_result;

static int write_full(int fd, const void* p, size_t n) {
  size_t off = 0;
  while (off < n) {
    ssize_t k = write(fd, (const char*)p + off, n - off);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) return -1;
    off += (size_t)k;
  }
  return 0;
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

/* a GPU context with the seeded registry and the message; reg (N*128) out */
static hg_ctx* setup_context(const opts* o, int p, uint8_t* reg, uint64_t* sk) {
  hg_ctx* ctx = NULL;
  if (A.create(0, HG_FLAVOR_GO, &ctx) != HG_OK) {
    fprintf(stderr, "proc %d: hg_create failed\n", p);
    child_exit(4);
  }
  if (o->level != -1) A.set_level(ctx, o->level);
  if (o->budget_mb >= 0) A.set_budget(ctx, (size_t)o->budget_mb << 20);
  const size_t N = (size_t)o->nreg;
  uint8_t* skb = (uint8_t*)malloc(N * 32);
  registry_secrets(o->nreg, sk, skb);
  int rc = A.set_message(ctx, kMsg, MSG_LEN);
  if (rc == HG_OK) rc = A.keygen(ctx, skb, N, reg);
  if (rc == HG_OK) rc = A.registry_load(ctx, reg, N, NULL);
  free(skb);
  if (rc != HG_OK) {
    fprintf(stderr, "proc %d: setup rc %d: %s\n", p, rc, A.last_error(ctx));
    child_exit(4);
  }
  return ctx;
}

static void sign_checks(hg_ctx* ctx, int p) {
  const size_t nchk = W_.nchk;
  int rc = A.sign(ctx, W_.agg_sk + (size_t)p * nchk * 32, nchk, W_.sigs + (size_t)p * nchk * 64);
  if (rc != HG_OK) {
    fprintf(stderr, "proc %d: sign rc %d: %s\n", p, rc, A.last_error(ctx));
    child_exit(4);
  }
}

/* ---------------------------------------------------------------- model 0: a context per process */
static hg_batcher* g_b;
static const opts* g_o;
static int g_p;
static int g_fail;

static void* batcher_worker(void* arg) {
  const int w = (int)(intptr_t)arg;
  const opts* o = g_o;
  check* chk = W_.checks + (size_t)g_p * W_.nchk;
  const uint64_t* words = W_.words + (size_t)g_p * W_.cap_words;
  const uint8_t* sigs = W_.sigs + (size_t)g_p * W_.nchk * 64;
  double* lat = W_.lat + (size_t)g_p * W_.nchk;
  /* instances w, w + W, w + 2W, ... of this process; one check each in flight */
  int mine = 0;
  for (int i = w; i < o->inst; i += o->workers) mine++;
  hg_ticket** t = (hg_ticket**)calloc((size_t)mine, sizeof(hg_ticket*));
  double* ts = (double*)calloc((size_t)mine, sizeof(double));
  for (int step = 0; step < o->checks; step++) {
    int j = 0;
    for (int i = w; i < o->inst; i += o->workers, j++) {
      const size_t k = (size_t)i * o->checks + step;
      ts[j] = now_s();
      if (A.b_submit(g_b, kMsg, MSG_LEN, &chk[k].req, words + chk[k].word_off, sigs + 64 * k, &t[j]) != HG_OK)
        g_fail = 1;
    }
    j = 0;
    for (int i = w; i < o->inst; i += o->workers, j++) {
      const size_t k = (size_t)i * o->checks + step;
      int32_t code = -1;
      if (A.b_wait(g_b, t[j], &code) != HG_OK) g_fail = 1;
      lat[k] = now_s() - ts[j];
      chk[k].got = code;
    }
  }
  free(t);
  free(ts);
  return NULL;
}

static void run_context_process(const opts* o, int p, int ready_fd, int start_fd, int out_fd) {
  proc_result res;
  memset(&res, 0, sizeof res);
  g_o = o;
  g_p = p;
  stage("process", p, "forked");
  resolve_gpu(o->lib);
  stage("process", p, "libhandel_gpu.so loaded");
  const double ts0 = now_s();
  const size_t N = (size_t)o->nreg;
  uint64_t* sk = (uint64_t*)malloc(N * 4 * sizeof(uint64_t));
  uint8_t* reg = (uint8_t*)malloc(N * 128);
  hg_ctx* ctx = setup_context(o, p, reg, sk);
  stage("process", p, "context, message, registry");
  gen_checks(o, p, sk, 0);
  sign_checks(ctx, p);
  stage("process", p, "checks signed");
  if (p == 0 && o->dump) {
    char path[4096];
    snprintf(path, sizeof path, "%s/reg.bin", o->dump);
    FILE* f = fopen(path, "wb");
    if (!f || fwrite(reg, 1, N * 128, f) != N * 128) res.rc = 1;
    if (f) fclose(f);
  }
  res.setup_s = now_s() - ts0;
  res.tables_before = A.tables(ctx);
  if (o->prepare) {
    const double tp = now_s();
    if (A.prepare(ctx) != HG_OK) {
      fprintf(stderr, "proc %d: prepare: %s\n", p, A.last_error(ctx));
      child_exit(4);
    }
    res.prepare_s = now_s() - tp;
    stage("process", p, "tables prepared");
  }
  if (A.b_create(ctx, (size_t)o->max_batch, (unsigned)o->wait_us, &g_b) != HG_OK) child_exit(4);
  char c1 = 'r';
  if (write(ready_fd, &c1, 1) != 1) child_exit(5);
  if (read(start_fd, &c1, 1) != 1) child_exit(5);
  stage("process", p, "started");
  pthread_t th[256];
  res.t0 = now_s();
  for (int w = 0; w < o->workers; w++) pthread_create(&th[w], NULL, batcher_worker, (void*)(intptr_t)w);
  for (int w = 0; w < o->workers; w++) pthread_join(th[w], NULL);
  res.t1 = now_s();
  stage("process", p, "checks done");
  A.b_stats(g_b, &res.batches, &res.requests);
  A.b_destroy(g_b);
  res.in_flight = 1;
  res.tables_after = A.tables(ctx);
  res.ctx_bytes = A.ctx_bytes(ctx);
  res.rc |= g_fail;
  A.destroy(ctx);
  stage("process", p, "context destroyed");
  if (write_full(out_fd, &res, sizeof res)) child_exit(5);
  child_exit(0);
}

/* ---------------------------------------------------------------- model 1: the verifier service */
static void service_name(char* buf, size_t cap, pid_t parent) { snprintf(buf, cap, "/hg_proxy_%d", (int)parent); }

static void run_server(const opts* o, pid_t parent, int ready_fd, int stop_fd, int out_fd) {
  proc_result res;
  memset(&res, 0, sizeof res);
  if (o->queues > 0) {
    char q[16];
    snprintf(q, sizeof q, "%d", o->queues);
    setenv("GPU_MAX_HW_QUEUES", q, 1); /* before the HIP runtime starts */
  }
  resolve_gpu(o->lib);
  char name[64];
  service_name(name, sizeof name, parent);
  hg_service_config cfg;
  A.s_config_init(&cfg);
  cfg.lanes = (uint32_t)o->lanes;
  cfg.max_batch = (uint32_t)o->max_batch;
  cfg.max_wait_us = (uint32_t)o->wait_us;
  cfg.quiet_us = (uint32_t)o->quiet_us;
  cfg.follow = o->follow;
  cfg.prepare = o->prepare;
  cfg.overlap = o->overlap;
  cfg.slot_bits = (uint32_t)o->nreg;
  hg_service* svc = NULL;
  hg_ctx* ctx = NULL;
  const double ts0 = now_s();
  const size_t N = (size_t)o->nreg;
  if (o->echo_us >= 0) {
    for (int p = 0; p < o->procs; p++) gen_checks(o, p, NULL, 1);
    res.setup_s = now_s() - ts0;
    if (A.s_create_echo(name, &cfg, (uint32_t)o->nreg, (uint32_t)o->echo_us, &svc) != HG_OK) {
      fprintf(stderr, "server: hg_service_create_echo failed\n");
      child_exit(4);
    }
  } else {
    uint64_t* sk = (uint64_t*)malloc(N * 4 * sizeof(uint64_t));
    uint8_t* reg = (uint8_t*)malloc(N * 128);
    ctx = setup_context(o, 0, reg, sk);
    for (int p = 0; p < o->procs; p++) {
      gen_checks(o, p, sk, 0);
      sign_checks(ctx, p);
    }
    if (o->dump) {
      char path[4096];
      snprintf(path, sizeof path, "%s/reg.bin", o->dump);
      FILE* f = fopen(path, "wb");
      if (!f || fwrite(reg, 1, N * 128, f) != N * 128) res.rc = 1;
      if (f) fclose(f);
    }
    res.setup_s = now_s() - ts0;
    res.tables_before = A.tables(ctx);
    if (o->prepare) {
      const double tp = now_s();
      if (A.prepare(ctx) != HG_OK) {
        fprintf(stderr, "server: prepare: %s\n", A.last_error(ctx));
        child_exit(4);
      }
      res.prepare_s = now_s() - tp;
    }
    if (A.s_create(ctx, name, &cfg, &svc) != HG_OK) {
      fprintf(stderr, "server: hg_service_create failed: %s\n", A.last_error(ctx));
      child_exit(4);
    }
  }
  char c1 = 'r';
  if (write(ready_fd, &c1, 1) != 1) child_exit(5);
  if (read(stop_fd, &c1, 1) != 1) res.rc = 1; /* the parent: every client is done */
  A.s_stats(svc, &res.batches, &res.requests, &res.in_flight);
  A.s_destroy(svc);
  if (ctx) {
    res.tables_after = A.tables(ctx);
    res.ctx_bytes = A.ctx_bytes(ctx);
    A.destroy(ctx);
  }
  if (write_full(out_fd, &res, sizeof res)) child_exit(5);
  child_exit(0);
}

typedef struct {
  int p, w;
  hg_client* cl;
  int fail;
} poller_arg;

static void* poller(void* arg) {
  poller_arg* a = (poller_arg*)arg;
  const opts* o = g_o;
  const int p = a->p;
  check* chk = W_.checks + (size_t)p * W_.nchk;
  const uint64_t* words = W_.words + (size_t)p * W_.cap_words;
  const uint8_t* sigs = W_.sigs + (size_t)p * W_.nchk * 64;
  double* lat = W_.lat + (size_t)p * W_.nchk;
  int mine = 0;
  for (int i = a->w; i < o->inst; i += o->workers) mine++;
  int* inst = (int*)calloc((size_t)mine, sizeof(int));
  int* step = (int*)calloc((size_t)mine, sizeof(int));
  uint64_t* tk = (uint64_t*)calloc((size_t)mine, sizeof(uint64_t));
  double* ts = (double*)calloc((size_t)mine, sizeof(double));
  int j = 0;
  for (int i = a->w; i < o->inst; i += o->workers) inst[j++] = i;
  /* every instance's first check, then one new check per verdict */
  for (j = 0; j < mine; j++) {
    const size_t k = (size_t)inst[j] * o->checks;
    ts[j] = now_s();
    if (C.submit(a->cl, kMsg, MSG_LEN, &chk[k].req, words + chk[k].word_off, sigs + 64 * k, &tk[j]) != HG_OK)
      a->fail = 1;
  }
  long left = (long)mine * o->checks;
  uint64_t got_t[512];
  int32_t got_c[512];
  while (left > 0 && !a->fail) {
    const int n = C.wait_any(a->cl, got_t, got_c, 512, 5000000);
    if (n <= 0) {
      fprintf(stderr, "proc %d poller %d: wait_any returned %d with %ld checks left\n", p, a->w, n, left);
      a->fail = 1;
      break;
    }
    const double t = now_s();
    for (int q = 0; q < n; q++) {
      int jj = 0;
      while (jj < mine && tk[jj] != got_t[q]) jj++;
      if (jj == mine) {
        a->fail = 1;
        continue;
      }
      const size_t k = (size_t)inst[jj] * o->checks + (size_t)step[jj];
      lat[k] = t - ts[jj];
      chk[k].got = got_c[q];
      left--;
      tk[jj] = 0;
      if (++step[jj] < o->checks) {
        const size_t k2 = k + 1;
        ts[jj] = now_s();
        if (C.submit(a->cl, kMsg, MSG_LEN, &chk[k2].req, words + chk[k2].word_off, sigs + 64 * k2, &tk[jj]) !=
            HG_OK)
          a->fail = 1;
      }
    }
  }
  free(inst);
  free(step);
  free(tk);
  free(ts);
  return NULL;
}

static void run_client_process(const opts* o, int p, pid_t parent, int ready_fd, int start_fd, int out_fd) {
  proc_result res;
  memset(&res, 0, sizeof res);
  g_o = o;
  resolve_client(o->client_lib);
  char name[64];
  service_name(name, sizeof name, parent);
  poller_arg pa[256];
  for (int w = 0; w < o->workers; w++) {
    pa[w].p = p;
    pa[w].w = w;
    pa[w].fail = 0;
    if (C.open(name, &pa[w].cl) != HG_OK) {
      fprintf(stderr, "client %d: hg_client_open(%s) failed\n", p, name);
      child_exit(4);
    }
  }
  char c1 = 'r';
  if (write(ready_fd, &c1, 1) != 1) child_exit(5);
  if (read(start_fd, &c1, 1) != 1) child_exit(5);
  pthread_t th[256];
  res.t0 = now_s();
  for (int w = 0; w < o->workers; w++) pthread_create(&th[w], NULL, poller, &pa[w]);
  for (int w = 0; w < o->workers; w++) pthread_join(th[w], NULL);
  res.t1 = now_s();
  for (int w = 0; w < o->workers; w++) {
    res.rc |= pa[w].fail;
    C.close(pa[w].cl);
  }
  res.requests = W_.nchk;
  if (write_full(out_fd, &res, sizeof res)) child_exit(5);
  child_exit(0);
}

/* ---------------------------------------------------------------- parent */
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

static int dump_process0(const opts* o) {
  const size_t nchk = W_.nchk;
  hg_request* rq = (hg_request*)malloc(nchk * sizeof(hg_request));
  int32_t* got = (int32_t*)malloc(nchk * sizeof(int32_t));
  size_t nwords = 0;
  for (size_t k = 0; k < nchk; k++) {
    rq[k] = W_.checks[k].req;
    got[k] = W_.checks[k].got;
    const size_t e = (size_t)W_.checks[k].word_off + W_.checks[k].nw;
    if (e > nwords) nwords = e;
  }
  int bad = write_file(o->dump, "reqs.bin", rq, nchk * sizeof(hg_request)) ||
            write_file(o->dump, "words.bin", W_.words, nwords * 8) ||
            write_file(o->dump, "sigs.bin", W_.sigs, nchk * 64) || write_file(o->dump, "codes.bin", got, nchk * 4);
  free(rq);
  free(got);
  return bad;
}

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: %s <libhandel_gpu.so> [-p P] [-k K] [-n N] [-r R] [-w W] [-b B] [-u U] [-P 0|1] "
                    "[-L level] [-M MB] [-D 0|1] [-l lanes] [-o 0|1] [-Q queues] [-q us] [-F 0|1] [-E us] [-C client.so] "
                    "[-d DIR]\n",
            argv[0]);
    return 2;
  }
  opts o = {8, 250, 2000, 45, -1, 4096, -1, 0, -1, 0, 8, 1, 0, 0, -1, -1, 1, NULL, argv[1], NULL};
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
    else if (!strcmp(f, "-D")) o.daemon = atoi(v);
    else if (!strcmp(f, "-l")) o.lanes = atoi(v);
    else if (!strcmp(f, "-o")) o.overlap = atoi(v);
    else if (!strcmp(f, "-Q")) o.queues = atoi(v);
    else if (!strcmp(f, "-q")) o.quiet_us = atoi(v);
    else if (!strcmp(f, "-F")) o.follow = atoi(v);
    else if (!strcmp(f, "-E")) o.echo_us = atol(v);
    else if (!strcmp(f, "-C")) o.client_lib = v;
    else if (!strcmp(f, "-d")) o.dump = v;
    else {
      fprintf(stderr, "unknown option %s\n", f);
      return 2;
    }
  }
  if (o.echo_us >= 0) o.daemon = 1;
  if (o.workers < 0) o.workers = o.daemon ? (o.inst >= 4 ? 4 : o.inst) : 16;
  if (o.daemon && o.queues == 0 && o.echo_us < 0) o.queues = 2 * o.lanes <= 32 ? 2 * o.lanes : 32;
  if (o.wait_us < 0) o.wait_us = o.daemon ? 50 : 200;
  static char client_path[4096];
  if (o.daemon && !o.client_lib) {
    const char* slash = strrchr(o.lib, '/');
    const int dl = slash ? (int)(slash - o.lib + 1) : 0;
    snprintf(client_path, sizeof client_path, "%.*slibhandel_client.so", dl, o.lib);
    o.client_lib = client_path;
  }
  if (o.procs < 1 || o.procs > 15 || o.inst < 1 || o.nreg < 2 || o.checks < 1 || o.workers < 1 ||
      o.workers > 256 || o.workers > o.inst || o.max_batch < 1 || o.lanes < 1 || o.lanes > 64 || o.queues < 0 ||
      o.queues > 32) {
    fprintf(stderr, "bad options (1 <= procs <= 15, 1 <= workers <= min(256, instances), 1 <= lanes <= 64, "
                    "queues <= 32)\n");
    return 2;
  }
  g_t_start = now_s();
  workload_map(&o);
  const pid_t me = getpid();
  pid_t pid[16], spid = -1;
  int ready[16][2], start[16][2], out[16][2];
  int sready[2], sstop[2], sout[2];
  if (o.daemon) {
    if (pipe(sready) || pipe(sstop) || pipe(sout)) return 6;
    spid = fork();
    if (spid < 0) return 6;
    if (spid == 0) {
      close(sready[0]);
      close(sstop[1]);
      close(sout[0]);
      run_server(&o, me, sready[1], sstop[0], sout[1]);
    }
    close(sready[1]);
    close(sstop[0]);
    close(sout[1]);
    char c;
    if (read_full(sready[0], &c, 1)) {
      fprintf(stderr, "handel_proxy: the server failed to start\n");
      waitpid(spid, NULL, 0);
      return 1;
    }
  }
  for (int p = 0; p < o.procs; p++) {
    if (pipe(ready[p]) || pipe(start[p]) || pipe(out[p])) return 6;
    pid[p] = fork();
    if (pid[p] < 0) return 6;
    if (pid[p] == 0) {
      close(ready[p][0]);
      close(start[p][1]);
      close(out[p][0]);
      if (o.daemon) run_client_process(&o, p, me, ready[p][1], start[p][0], out[p][1]);
      else run_context_process(&o, p, ready[p][1], start[p][0], out[p][1]);
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
  stage("parent", 0, "every process ready");
  for (int p = 0; p < o.procs; p++) {
    char c = 's';
    if (write(start[p][1], &c, 1) != 1) bad = 1;
  }
  proc_result r[16], srv;
  memset(&srv, 0, sizeof srv);
  for (int p = 0; p < o.procs; p++) {
    if (read_full(out[p][0], &r[p], sizeof r[p])) {
      fprintf(stderr, "process %d: no result\n", p);
      bad = 1;
      memset(&r[p], 0, sizeof r[p]);
    }
  }
  stage("parent", 0, "every result in");
  for (int p = 0; p < o.procs; p++) {
    int st = 0;
    waitpid(pid[p], &st, 0);
    if (!WIFEXITED(st) || WEXITSTATUS(st) != 0) bad = 1;
  }
  stage("parent", 0, "every process exited");
  if (o.daemon) {
    char c = 'q';
    if (write(sstop[1], &c, 1) != 1) bad = 1;
    if (read_full(sout[0], &srv, sizeof srv)) {
      fprintf(stderr, "server: no result\n");
      bad = 1;
    }
    int st = 0;
    waitpid(spid, &st, 0);
    if (!WIFEXITED(st) || WEXITSTATUS(st) != 0) bad = 1;
  }
  if (bad) {
    fprintf(stderr, "handel_proxy: a process failed\n");
    return 1;
  }
  const size_t nchk = W_.nchk, m = nchk * (size_t)o.procs;
  double t0 = r[0].t0, t1 = r[0].t1, setup = srv.setup_s, prep = srv.prepare_s;
  uint64_t reqs = 0, batches = srv.batches, mism = 0, bytes_max = srv.ctx_bytes, bytes_all = srv.ctx_bytes;
  uint64_t in_flight = srv.in_flight;
  int fails = srv.rc, tb = o.daemon ? srv.tables_before : r[0].tables_before;
  int ta = o.daemon ? srv.tables_after : r[0].tables_after;
  for (int p = 0; p < o.procs; p++) {
    if (r[p].t0 < t0) t0 = r[p].t0;
    if (r[p].t1 > t1) t1 = r[p].t1;
    if (r[p].setup_s > setup) setup = r[p].setup_s;
    if (r[p].prepare_s > prep) prep = r[p].prepare_s;
    if (r[p].ctx_bytes > bytes_max) bytes_max = r[p].ctx_bytes;
    bytes_all += r[p].ctx_bytes;
    if (!o.daemon) {
      reqs += r[p].requests;
      batches += r[p].batches;
    }
    fails += r[p].rc;
  }
  if (o.daemon) reqs = srv.requests;
  for (size_t k = 0; k < m; k++) mism += W_.checks[k].got != W_.checks[k].expect;
  if (o.dump && dump_process0(&o)) fails++;
  double* lat = (double*)malloc(m * sizeof(double));
  memcpy(lat, W_.lat, m * sizeof(double));
  qsort(lat, m, sizeof(double), cmp_double);
  const double wall = t1 - t0;
  printf("{\"harness\": \"handel_proxy\", \"what\": \"config-4 process-model proxy (not Handel completion time)\", "
         "\"model\": \"%s\", \"procs\": %d, \"instances_per_proc\": %d, \"nodes\": %d, \"registry\": %d, "
         "\"checks_per_instance\": %d, \"workers_per_proc\": %d, \"prepare\": %d, \"lanes\": %d, \"overlap\": %d, "
         "\"hw_queues\": %d, \"max_wait_us\": %d, \"quiet_us\": %d, \"follow\": %d, \"echo_us\": %ld, \"tables_before\": %d, \"tables_after\": %d, "
         "\"requests\": %llu, \"batches\": %llu, \"mean_batch\": %.1f, \"max_batches_in_flight\": %llu, "
         "\"wall_ms\": %.3f, \"throughput\": %.1f, "
         "\"latency_us\": {\"p50\": %.1f, \"p90\": %.1f, \"p99\": %.1f, \"max\": %.1f}, "
         "\"hbm_per_context_bytes\": %llu, \"hbm_total_bytes\": %llu, \"contexts\": %d, "
         "\"setup_s_max\": %.3f, \"prepare_ms_max\": %.3f, \"mismatches\": %llu}\n",
         o.daemon ? (o.echo_us >= 0 ? "daemon-echo" : "daemon") : "contexts", o.procs, o.inst, o.procs * o.inst,
         o.nreg, o.checks, o.workers, o.prepare, o.daemon ? o.lanes : 1, o.overlap, o.queues, o.wait_us, o.quiet_us, o.follow, o.echo_us,
         tb, ta, (unsigned long long)reqs, (unsigned long long)batches, batches ? (double)reqs / batches : 0.0,
         (unsigned long long)in_flight, wall * 1e3, wall > 0 ? reqs / wall : 0.0, 1e6 * lat[m / 2],
         1e6 * lat[(m * 9) / 10], 1e6 * lat[(m * 99) / 100], 1e6 * lat[m - 1], (unsigned long long)bytes_max,
         (unsigned long long)bytes_all, o.daemon ? (o.echo_us >= 0 ? 0 : 1) : o.procs, setup, prep * 1e3,
         (unsigned long long)mism);
  free(lat);
  return (mism || fails || reqs != m) ? 1 : 0;
}
