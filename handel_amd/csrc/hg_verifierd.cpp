// hg_verifierd — the GPU-owning verifier process of a single-host simul run
// (simul/node/main.go:63-131: P OS processes of k Handel instances each). It
// owns the GPU context, decodes the run's registry once, builds the GT tables
// of the run's message once, and serves every client process through the
// shared-memory region `--name` (hg_service_*; clients link only
// libhandel_client.so, include/handel_client.h). Runs until SIGINT/SIGTERM,
// then verifies what is queued, prints one JSON line of statistics and exits.
//
//   hg_verifierd --name /handel --registry reg.bin [--flavor go|cf] [--device 0]
//                [--message msg.bin] [--lanes 8] [--max-batch 4096]
//                [--max-wait-us 50] [--quiet-us 0] [--follow 1] [--policy] [--overlap 1]
//   hg_verifierd --name /handel --echo US --nreg N      (CPU stand-in, no GPU)
//
// reg.bin: n x 128-byte marshalled public keys in registry order
// (PublicKey.MarshalBinary, bn256/go/bn256.go:107-111). msg.bin: the run's
// message (lib.Message); with it the tables are built before "ready" is
// printed, otherwise at the first request. --policy: the volume policy
// instead of building the top table level at a message's first batch.
#include <pthread.h>

#include <csignal>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/handel_gpu.h"

namespace {

bool read_file(const char* path, std::vector<uint8_t>& out) {
  FILE* f = fopen(path, "rb");
  if (!f) return false;
  uint8_t buf[1 << 16];
  size_t k;
  while ((k = fread(buf, 1, sizeof buf, f)) > 0) out.insert(out.end(), buf, buf + k);
  const bool ok = !ferror(f);
  fclose(f);
  return ok;
}

int usage() {
  fprintf(stderr,
          "usage: hg_verifierd --name /NAME (--registry FILE | --echo US --nreg N) [--flavor go|cf] [--device D]\n"
          "                    [--message FILE] [--lanes L] [--max-batch B] [--max-wait-us U] [--quiet-us Q]\n"
          "                    [--follow 0|1] [--policy] [--overlap 0|1] [--slots S]\n");
  return 2;
}

}  // namespace

int main(int argc, char** argv) {
  const char *name = nullptr, *reg_path = nullptr, *msg_path = nullptr;
  int flavor = HG_FLAVOR_GO, device = 0;
  long echo_us = -1, nreg_echo = 0;
  hg_service_config cfg;
  hg_service_config_init(&cfg);
  for (int i = 1; i < argc; i++) {
    const std::string a = argv[i];
    const char* v = i + 1 < argc ? argv[i + 1] : nullptr;
    auto need = [&]() -> const char* {
      if (!v) exit(usage());
      i++;
      return v;
    };
    if (a == "--name") name = need();
    else if (a == "--registry") reg_path = need();
    else if (a == "--message") msg_path = need();
    else if (a == "--flavor") {
      const std::string f = need();
      if (f == "go" || f == "bn256/go") flavor = HG_FLAVOR_GO;
      else if (f == "cf" || f == "bn256/cf" || f == "bn256") flavor = HG_FLAVOR_CF;
      else return usage();
    } else if (a == "--device") device = atoi(need());
    else if (a == "--lanes") cfg.lanes = (uint32_t)atoi(need());
    else if (a == "--max-batch") cfg.max_batch = (uint32_t)atoi(need());
    else if (a == "--max-wait-us") cfg.max_wait_us = (uint32_t)atoi(need());
    else if (a == "--quiet-us") cfg.quiet_us = (uint32_t)atoi(need());
    else if (a == "--slots") cfg.slots = (uint32_t)atoi(need());
    else if (a == "--overlap") cfg.overlap = atoi(need());
    else if (a == "--follow") cfg.follow = atoi(need());
    else if (a == "--policy") cfg.prepare = 0;
    else if (a == "--echo") echo_us = atol(need());
    else if (a == "--nreg") nreg_echo = atol(need());
    else return usage();
  }
  if (!name || (echo_us < 0 && !reg_path) || (echo_us >= 0 && nreg_echo <= 0)) return usage();

  // each lane runs on two streams (the pairing kernel, the fold beside it):
  // one hardware queue per stream, unless the environment says otherwise
  // (read when the HIP runtime starts, below; more than ~16 queues per process
  // measured slower: profiles/r04_proxy_sweep.jsonl)
  if (echo_us < 0 && !getenv("GPU_MAX_HW_QUEUES")) {
    const unsigned q = 2 * cfg.lanes < 32 ? 2 * cfg.lanes : 32;
    setenv("GPU_MAX_HW_QUEUES", std::to_string(q).c_str(), 1);
  }
  // the signals that end the service are taken synchronously below
  sigset_t stop;
  sigemptyset(&stop);
  sigaddset(&stop, SIGINT);
  sigaddset(&stop, SIGTERM);
  pthread_sigmask(SIG_BLOCK, &stop, nullptr);  // before any thread starts

  hg_ctx* ctx = nullptr;
  hg_service* svc = nullptr;
  size_t nreg = 0;
  if (echo_us >= 0) {
    nreg = (size_t)nreg_echo;
    if (hg_service_create_echo(name, &cfg, (uint32_t)nreg, (uint32_t)echo_us, &svc) != HG_OK) {
      fprintf(stderr, "hg_verifierd: cannot create %s\n", name);
      return 1;
    }
  } else {
    std::vector<uint8_t> reg, msg;
    if (!read_file(reg_path, reg) || reg.empty() || reg.size() % 128) {
      fprintf(stderr, "hg_verifierd: %s: not a list of 128-byte keys\n", reg_path);
      return 2;
    }
    if (msg_path && !read_file(msg_path, msg)) {
      fprintf(stderr, "hg_verifierd: cannot read %s\n", msg_path);
      return 2;
    }
    nreg = reg.size() / 128;
    if (hg_create(device, flavor, &ctx) != HG_OK) {
      fprintf(stderr, "hg_verifierd: no GPU context on device %d\n", device);
      return 1;
    }
    std::vector<int32_t> codes(nreg);
    if (hg_registry_load(ctx, reg.data(), nreg, codes.data()) != HG_OK) {
      size_t bad = 0;
      while (bad < nreg && codes[bad] == HG_OK) bad++;
      fprintf(stderr, "hg_verifierd: registry key %zu: %s\n", bad, hg_code_string(codes[bad < nreg ? bad : 0], flavor));
      hg_destroy(ctx);
      return 3;
    }
    if (msg_path) {
      const int rc = cfg.prepare ? hg_prepare_aggregate_msg(ctx, msg.data(), msg.size())
                                 : hg_set_message(ctx, msg.data(), msg.size());
      if (rc != HG_OK && rc != HG_ERR_HASH_EOF) {
        fprintf(stderr, "hg_verifierd: message setup: %s\n", hg_last_error(ctx));
        hg_destroy(ctx);
        return 1;
      }
    }
    if (hg_service_create(ctx, name, &cfg, &svc) != HG_OK) {
      fprintf(stderr, "hg_verifierd: cannot create %s: %s\n", name, hg_last_error(ctx));
      hg_destroy(ctx);
      return 1;
    }
  }
  printf("{\"ready\": \"%s\", \"registry\": %zu, \"lanes\": %u, \"tables\": %d}\n", name, nreg, cfg.lanes,
         ctx ? hg_aggregate_tables(ctx) : 0);
  fflush(stdout);
  int sig = 0;
  sigwait(&stop, &sig);
  uint64_t batches = 0, requests = 0, in_flight = 0;
  hg_service_stats(svc, &batches, &requests, &in_flight);
  hg_service_destroy(svc);  // verifies what is still queued
  printf("{\"stopped\": \"%s\", \"signal\": %d, \"batches\": %llu, \"requests\": %llu, \"max_batches_in_flight\": %llu, "
         "\"tables\": %d, \"device_bytes\": %zu}\n",
         name, sig, (unsigned long long)batches, (unsigned long long)requests, (unsigned long long)in_flight,
         ctx ? hg_aggregate_tables(ctx) : 0, ctx ? hg_context_bytes(ctx) : (size_t)0);
  fflush(stdout);
  if (ctx) hg_destroy(ctx);
  return 0;
}
