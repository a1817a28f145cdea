/*
 * handel_client.h — client side of the verifier service (hg_service_* in
 * handel_gpu.h). libhandel_client.so has no GPU or HIP dependency: a simul
 * process (simul/node/main.go:63-131) that runs k Handel instances attaches
 * to the service's shared-memory region by name and submits each instance's
 * aggregate check there instead of opening its own GPU context. A Go
 * maintainer binds it with cgo exactly like the hg_batcher_* entry points
 * (INTEGRATION.md); the request layout and codes are handel_gpu.h's.
 *
 * Thread safety: submit may be called from any thread; wait / wait_any may be
 * called from several threads of the same handle (one of them drains the
 * handle's completion ring at a time). Each handle owns one completion
 * channel of the region; open one handle per process (or per poller thread).
 */
#ifndef HANDEL_CLIENT_H
#define HANDEL_CLIENT_H

#include <stddef.h>
#include <stdint.h>

#include "handel_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct hg_client hg_client;

/* Attaches to the service region `name`; HG_ERR_ARG if it does not exist,
 * is not a running service, or has no free channel. */
int hg_client_open(const char* name, hg_client** out);
/* Releases the handle (tickets not yet collected are dropped: the service
 * frees their slots when they finish, and keeps the handle's channel reserved
 * until then, so no later handle receives their completions). Must not run
 * concurrently with submit / wait / wait_any on the same handle: stop the
 * threads that use it first. */
void hg_client_close(hg_client* cl);
/* Queues one processing.go verifySignature (:342-368): the level range
 * [req->offset, req->offset + req->level_size), the bitset of req->bitlen bits
 * at words (ceil(bitlen / 64) words, bit i = words[i >> 6] bit (i & 63)), the
 * 64-byte signature marshal, under message msg (req->word_offset is ignored).
 * Inputs are copied. *ticket identifies it for hg_client_wait; every ticket
 * is collected once (wait, or wait_any). HG_ERR_ARG: bad arguments, a bitset
 * longer than the region's slot_bits, a message longer than 1024 bytes, or
 * the service is stopping. */
int hg_client_submit(hg_client* cl, const uint8_t* msg, size_t len, const hg_request* req, const uint64_t* words,
                     const uint8_t* sig, uint64_t* ticket);
/* Blocks until the ticket's batch ran; *code = its hg_code. HG_OK, or
 * HG_ERR_ARG (unknown ticket) / HG_ERR_DEVICE (the service stopped first). */
int hg_client_wait(hg_client* cl, uint64_t ticket, int32_t* code);
/* Collects up to cap finished tickets of this handle (any order), waiting at
 * most timeout_us (< 0: no limit) for the first. Returns the count (0 on
 * timeout), or -HG_ERR_DEVICE once the service has stopped and nothing is
 * left to collect. */
int hg_client_wait_any(hg_client* cl, uint64_t* tickets, int32_t* codes, size_t cap, long timeout_us);
/* submit + wait. */
int hg_client_verify_aggregate(hg_client* cl, const uint8_t* msg, size_t len, const hg_request* req,
                               const uint64_t* words, const uint8_t* sig, int32_t* code);
/* The service's batches launched and requests verified so far. */
int hg_client_stats(hg_client* cl, uint64_t* batches, uint64_t* requests);
/* The region's largest bitset per request, in bits. */
uint32_t hg_client_slot_bits(hg_client* cl);
/* The service context's flavor, and the reference's texts for a code under
 * it: hg_code_string's and hg_processing_error_string's (processing.go:342-368:
 * VerifySignature's errors wrapped "handel: <err>"), without linking the GPU
 * library. */
int hg_client_flavor(hg_client* cl);
const char* hg_client_code_string(hg_client* cl, int code);
const char* hg_client_processing_error_string(hg_client* cl, int code);

#ifdef __cplusplus
}
#endif
#endif /* HANDEL_CLIENT_H */
