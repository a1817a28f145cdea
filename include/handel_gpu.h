/*
 * handel_gpu.h — C ABI of the MI355X BN256 BLS verification engine.
 *
 * This is the drop-in boundary for Handel's crypto plugin interfaces
 * (crypto.go:14-54: PublicKey / Signature / Constructor / MultiSignature)
 * on the bn256 path. A Go maintainer binds it with cgo;
 * the Python host package handel_amd binds it with ctypes. Plain pointers
 * and sizes only; every entry point is thread-safe per context (a mutex
 * serialises submitters, matching the concurrent Handel instances of
 * simul/node/main.go:63-77). Work submitted on one context runs in
 * submission order even across HIP streams: each asynchronous submission
 * records an event, and the next submission on another stream waits for it,
 * because the submissions share the context's device workspaces.
 *
 * Byte formats are the reference's marshals:
 *   G1 (signature)  64 B  = x || y, 32-byte big-endian affine coords, zeros = infinity
 *   G2 (public key) 128 B = x.x || x.y || y.x || y.y (x = x.x*i + x.y), zeros = infinity
 *   GT              384 B = x/crypto GT.Marshal order
 *   bitsets          willf/bitset words: bit i = word[i >> 6] bit (i & 63)
 */
#ifndef HANDEL_GPU_H
#define HANDEL_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Per-check result codes. Each maps 1:1 to the error the reference returns
 * (hg_code_string gives the exact text for the chosen flavor). */
enum hg_code {
  HG_OK = 0,                /* nil */
  HG_ERR_SIG_INVALID = 1,   /* "bn256: signature invalid"            bn256/go/bn256.go:91 */
  HG_ERR_HASH_EOF = 2,      /* "EOF" (hashedMessage, digest >= n)     bn256/go/bn256.go:210-218 */
  HG_ERR_LEVEL = 3,         /* "handel: inconsistent bitset with given level" processing.go:350-352 */
  HG_ERR_PK_UNMARSHAL = 4,  /* "unable to unmarshal"                  bn256/go/bn256.go:117 */
  HG_ERR_SIG_UNMARSHAL = 5, /* "bn256: multisig can't unmarshal"      bn256/go/bn256.go:186 */
  HG_ERR_EMPTY_AGG = 6,     /* empty bitset: the reference dereferences a nil *G2 (panic) */
  HG_ERR_CF_EXCEEDS = 7,    /* cloudflare: "bn256: coordinate exceeds modulus" */
  HG_ERR_CF_MALFORMED = 8,  /* cloudflare: "bn256: malformed point" */
  HG_ERR_CF_SHORT = 9,      /* cloudflare: "bn256: not enough data" */
  /* cloudflare SigBLS.UnmarshalBinary wraps the G1 error (bn256/cf/bn256.go:183-190) */
  HG_ERR_SIG_CF_EXCEEDS = 10,   /* "bn256: multisig can't unmarshal: bn256: coordinate exceeds modulus" */
  HG_ERR_SIG_CF_MALFORMED = 11, /* "bn256: multisig can't unmarshal: bn256: malformed point" */
  HG_ERR_SIG_CF_SHORT = 12,     /* "bn256: multisig can't unmarshal: bn256: not enough data" */
  HG_ERR_MULTI_SIZES = 13,  /* "verify multisignature: inconsistent sizes"  crypto.go:122-124 */
  /* Handel packet intake (hg_parse_packets): handel.go:371-436 validatePacket /
   * parseSignatures, crypto.go:86-110 MultiSignature.Unmarshal, bitset.go:166-177
   * WilffBitSet.UnmarshalBinary over willf/bitset v1.1.10 ReadFrom */
  HG_ERR_PKT_ORIGIN = 20,        /* "packet's origin out of range"              handel.go:374-376 */
  HG_ERR_PKT_LEVEL = 21,         /* "invalid packet's level %d"                 handel.go:378-383 */
  HG_ERR_PKT_EOF = 22,           /* "EOF" (encoding/binary.Read on no bytes)    crypto.go:89, bitset.go:169 */
  HG_ERR_PKT_UNEXPECTED_EOF = 23, /* "unexpected EOF" (binary.Read, short read) */
  HG_ERR_PKT_BITSET_SHORT = 24,  /* "bitset received smaller than expected"     crypto.go:93-96 */
  HG_ERR_PKT_TYPE_MISMATCH = 25, /* "unmarshalling error: type mismatch"        willf ReadFrom */
  HG_ERR_PKT_BITSET_SIZE = 26,   /* "invalid bitset's size for given level"     handel.go:398-401 */
  HG_ERR_PKT_NO_SIG = 27,        /* "no signature in the bitset"                handel.go:402-405 */
  HG_ERR_PKT_ID_RANGE = 28,      /* "globalID outside level's range. id=%d, min=%d, max=%d, level=%d"
                                    partitioner.go:107-119 IndexAtLevel, handel.go:421-425 */
  HG_PKT_NO_IND = 29,            /* not an error: the packet carried no individual signature */
  HG_ERR_ARG = 100,         /* bad argument to this API */
  HG_ERR_DEVICE = 101       /* HIP runtime failure (see hg_last_error) */
};

/* Which upstream library's Unmarshal rules to mirror (simul/lib/config.go:211-225). */
enum hg_flavor {
  HG_FLAVOR_GO = 0, /* golang.org/x/crypto/bn256  ("bn256/go") */
  HG_FLAVOR_CF = 1  /* github.com/cloudflare/bn256 ("bn256", "bn256/cf") */
};

typedef struct hg_ctx hg_ctx;

/* One aggregate-verification request (processing.go:342-368 verifySignature):
 * the level's registry range starts at `offset` (partitioner.go rangeLevel min),
 * `level_size` = max - min, the bitset has `bitlen` bits stored at
 * words[word_offset ...]. bitlen != level_size -> HG_ERR_LEVEL. */
typedef struct {
  uint32_t offset;
  uint32_t bitlen;
  uint32_t level_size;
  uint32_t word_offset;
} hg_request;

/* Context: owns a device, the decoded registry, the hashed message and the
 * precomputed G2Base line table. Replaces bn256.NewConstructor() + the
 * package-level G2Base (bn256/go/bn256.go:22,28-52). */
int hg_create(int device, int flavor, hg_ctx** out);
void hg_destroy(hg_ctx* ctx);
const char* hg_last_error(hg_ctx* ctx);
const char* hg_code_string(int code, int flavor);
/* The error text processing.go's verifySignature returns for a per-request
 * code (processing.go:342-368): VerifySignature's errors (signature invalid,
 * hash EOF) wrapped as "handel: <err>", the level check's own text unwrapped,
 * everything else as hg_code_string. "" for HG_OK. */
const char* hg_processing_error_string(int code, int flavor);
int hg_version(void);
/* The context's flavor (HG_FLAVOR_GO / HG_FLAVOR_CF), -1 for NULL. */
int hg_context_flavor(hg_ctx* ctx);
/* SIMDs of the context's device (compute units x 4): the pairing waves it
 * holds at one wave per SIMD (the padded kernels); 0 on error. */
int hg_context_simds(hg_ctx* ctx);

/* Registry.Identities(...).PublicKey() source: uploads n marshalled G2
 * public keys (PublicKey.UnmarshalBinary, bn256/go/bn256.go:113-120), decoding
 * them on the GPU. codes (nullable, n entries) receives per-key decode codes;
 * returns HG_OK only if every key decoded. On any failure the context is
 * left with NO registry (size 0): every aggregate request then fails its
 * range check instead of reading tables of another registry. */
int hg_registry_load(hg_ctx* ctx, const uint8_t* pks, size_t n, int32_t* codes);
size_t hg_registry_size(hg_ctx* ctx);

/* hashedMessage (bn256/go/bn256.go:210-218) computed once per message and
 * cached on the device. Returns HG_OK or HG_ERR_HASH_EOF. */
int hg_set_message(hg_ctx* ctx, const uint8_t* msg, size_t len);

/* PublicKey.VerifySignature(msg, sig) x n with the message given per call
 * (bn256/go/bn256.go:82-94): hashing (cached when msg equals the context's
 * current message) and verification happen under ONE lock hold, so
 * concurrent callers with different messages cannot interleave. */
int hg_verify_batch_msg(hg_ctx* ctx, const uint8_t* msg, size_t len, const uint8_t* pks, const uint8_t* sigs,
                        size_t n, int32_t* codes);

/* n independent PublicKey.VerifySignature(msg, sig) checks (bn256/go:82-94;
 * simul/p2p/aggregator.go:244). pks: n*128 B, sigs: n*64 B, codes: n. */
int hg_verify_batch(hg_ctx* ctx, const uint8_t* pks, const uint8_t* sigs, size_t n, int32_t* codes);

/* Same, with pks/sigs/codes already resident in device memory; `stream` is a
 * hipStream_t (NULL = the context's stream). Asynchronous on the stream. */
int hg_verify_batch_device(hg_ctx* ctx, const uint8_t* d_pks, const uint8_t* d_sigs, size_t n, int32_t* d_codes,
                           void* stream);

/* Verdict bitset of n device-resident codes: bit j of byte b (LSB first) = 1
 * iff check 8b+j returned HG_OK; ceil(n/8) bytes, tail bits 0. Replaces the
 * per-check `err == nil` branch of verifyAndPublish (processing.go:270-287)
 * with the buffer the multi-GPU gather exchanges. Asynchronous on `stream`. */
int hg_pack_verdicts_device(hg_ctx* ctx, const int32_t* d_codes, size_t n, uint8_t* d_bits, void* stream);

/* n aggregate checks against the registry: the Combine fold over the set
 * bits of each request's level range, then VerifySignature
 * (processing.go:342-368; crypto.go:120-137 for a full-registry request).
 * agg_pk_out (nullable): n*128 B marshal of each aggregate public key. */
int hg_verify_aggregate(hg_ctx* ctx, const hg_request* reqs, size_t n, const uint64_t* words, size_t nwords,
                        const uint8_t* sigs, int32_t* codes, uint8_t* agg_pk_out);

/* hg_verify_aggregate with the message given per call: hashing (cached when
 * msg equals the context's current message) and the batch under ONE lock
 * hold, for callers that share a context across messages. */
int hg_verify_aggregate_msg(hg_ctx* ctx, const uint8_t* msg, size_t len, const hg_request* reqs, size_t n,
                            const uint64_t* words, size_t nwords, const uint8_t* sigs, int32_t* codes,
                            uint8_t* agg_pk_out);

/* VerifyMultiSignature (crypto.go:120-137) x n: request i's bitset of
 * bitlens[i] bits at words[word_offsets[i] ...] must span the whole registry
 * (bitlens[i] != registry size -> HG_ERR_MULTI_SIZES, the reference's
 * "verify multisignature: inconsistent sizes"). The reference's "registry
 * returned empty identity" cannot occur: the registry is dense. */
int hg_verify_multisig(hg_ctx* ctx, const uint32_t* bitlens, const uint32_t* word_offsets, size_t n,
                       const uint64_t* words, size_t nwords, const uint8_t* sigs, int32_t* codes);

/* Builds the per-(message, registry) tables of aggregate verification now:
 * e(H, pk_i) for every registry key and the GT products of every 8-key and
 * 16-key window subset and aligned block (bilinearity: e(H, sum pk_i) =
 * prod e(H, pk_i); the aggregate check is then a GT fold plus ONE pairing per
 * request). For serving a stream of batches (≈ 15 ms and ≈ 2 MB of HBM per
 * key; registries above 16384 keys get the 8-key tables only). Without it the
 * context builds the 8-key level after 16384 requests of one message (≈ 3 ms
 * for 4000 keys) and the 16-key level after 2^20, verifying earlier requests
 * with the G2 point fold. Tables follow the context's current message and
 * registry. HG_OK; HG_ERR_HASH_EOF (message cannot be hashed: nothing to
 * build); HG_ERR_ARG without a message or registry. Synchronous. */
int hg_prepare_aggregate(hg_ctx* ctx);
/* hg_set_message + hg_prepare_aggregate under ONE lock hold, so a concurrent
 * caller with another message cannot take the tables in between (the Go
 * PrepareAggregate, bn256/go/bn256.go:210-218: H is fixed per Handel run). */
int hg_prepare_aggregate_msg(hg_ctx* ctx, const uint8_t* msg, size_t len);
/* The table level aggregate requests currently run at: 0 = G2 point fold and
 * two-pairing check, 1 = GT fold over 8-key windows, 2 = over 16-key windows.
 * The tables are a cache: a level the device cannot hold (or that exceeds the
 * table budget) is skipped and requests run at the level below, down to 0.
 * A go-flavor registry holding a key outside G2 stays at 0 (see
 * hg_registry_non_g2). */
int hg_aggregate_tables(hg_ctx* ctx);
/* Pins the table level of this context's aggregate submissions (0..2, capped
 * as above) or, with -1, returns them to the volume policy. New contexts take
 * HG_GT_LEVEL / HG_AGG_PATH=g2 (= 0) from the environment, else -1. */
int hg_set_aggregate_level(hg_ctx* ctx, int level);
/* GT path: run the fold on a side stream beside the pairing kernel (1, the
 * default; HG_GT_OVERLAP=0 makes 0 the default of new contexts) or before it
 * (0). Same verdicts; the overlap hides the fold when one batch is in flight,
 * several contexts each with a batch in flight may prefer 0. */
int hg_set_fold_overlap(hg_ctx* ctx, int on);
/* Config 2 (hg_verify_batch*): the check's form. 0 (the default; HG_VERIFY_SPLIT
 * gives new contexts its value): one kernel per batch, the faster form when a
 * batch runs alone. 1: the split form — the Miller loop on a compact team
 * region, then the 12-lane final exponentiation with batched inversions — for
 * several contexts each keeping a batch in flight, whose waves then share the
 * SIMDs. Same verdicts (PublicKey.VerifySignature, bn256/go/bn256.go:82-94). */
int hg_set_verify_split(hg_ctx* ctx, int on);
/* Upper bound in bytes for this context's GT tables (default: unlimited, the
 * device's free memory decides). Processes sharing one GPU (simul's P
 * processes x k instances, simul/node/main.go:63-131) give each context a
 * share; level-2 tables take ~1.97 MB per key, level 1 ~15 kB per key. */
int hg_set_table_budget(hg_ctx* ctx, size_t bytes);
/* Keys of the loaded registry that lie on the twist but outside the order-n
 * subgroup G2. x/crypto's G2.Unmarshal accepts them (bn256/go/bn256.go:113-120;
 * cloudflare rejects them at load). The GT product e(H, pk_1)...e(H, pk_k)
 * equals the reference's e(H, pk_1 + ... + pk_k) only on G2, so a registry
 * with such keys is served by the G2 fold and the two-pairing check. */
size_t hg_registry_non_g2(hg_ctx* ctx);

/* Device-resident variant (reqs, words, sigs, codes, agg out on the device). */
int hg_verify_aggregate_device(hg_ctx* ctx, const hg_request* d_reqs, size_t n, const uint64_t* d_words,
                               const uint8_t* d_sigs, int32_t* d_codes, uint8_t* d_agg_pk_out, void* stream);

/* hg_verify_aggregate_device (verdicts only) plus the verdict bitset of the
 * codes (hg_pack_verdicts_device's layout, ceil(n/8) bytes) in the same
 * submission: the serving step's codes -> bitset launch folds into the
 * comparison (processing.go:270-287's err == nil branch, batched). */
int hg_verify_aggregate_device_bits(hg_ctx* ctx, const hg_request* d_reqs, size_t n, const uint64_t* d_words,
                                    const uint8_t* d_sigs, int32_t* d_codes, uint8_t* d_bits, void* stream);

/* Batched PublicKey.Combine fold only: n requests -> n*128 B aggregate keys
 * (bn256/go/bn256.go:97-105). codes: HG_OK, HG_ERR_LEVEL or HG_ERR_EMPTY_AGG. */
int hg_aggregate_pk(hg_ctx* ctx, const hg_request* reqs, size_t n, const uint64_t* words, size_t nwords,
                    uint8_t* agg_pk_out, int32_t* codes);

/* Batched SigBLS.Combine (bn256/go/bn256.go:192-200): out[i] = a[i] + b[i]. */
int hg_combine_g1(hg_ctx* ctx, const uint8_t* a, const uint8_t* b, size_t n, uint8_t* out, int32_t* codes);

/* Batched PublicKey.Combine on marshalled keys (bn256/go/bn256.go:97-105):
 * out[i] = a[i] + b[i] in G2 (n*128 B each). */
int hg_combine_g2(hg_ctx* ctx, const uint8_t* a, const uint8_t* b, size_t n, uint8_t* out, int32_t* codes);

/* bn256.Pair(g1[i], g2[i]).Marshal() — the GT values the reference compares
 * in VerifySignature (bn256/go/bn256.go:88-89); parity probe. */
int hg_pair(hg_ctx* ctx, const uint8_t* g1s, const uint8_t* g2s, size_t n, uint8_t* gt_out, int32_t* codes);

/* Batch keygen / signing for fixtures and simulation start-up:
 * NewKeyPair's pk = k * G2 (bn256/go/bn256.go:129-142) and Sign's
 * sig = k * H(msg) (bn256/go/bn256.go:146-154) for n big-endian 32-byte
 * scalars. hg_sign needs hg_set_message first (returns HG_ERR_HASH_EOF when
 * the message cannot be hashed). */
int hg_keygen(hg_ctx* ctx, const uint8_t* scalars_be, size_t n, uint8_t* pks_out);
int hg_sign(hg_ctx* ctx, const uint8_t* scalars_be, size_t n, uint8_t* sigs_out);
/* SecretKey.Sign(msg) x n with the message given per call (one lock hold,
 * like hg_verify_batch_msg). */
int hg_sign_msg(hg_ctx* ctx, const uint8_t* msg, size_t len, const uint8_t* scalars_be, size_t n,
                uint8_t* sigs_out);

/* Self test of the field multiplier: out = a*b mod p on plain 256-bit
 * little-endian 32-bit words (8 per element). */
int hg_debug_fp_mul(hg_ctx* ctx, const uint32_t* a, const uint32_t* b, size_t n, uint32_t* out);

/* Measurement hooks: when enabled, device work is bracketed by HIP events on
 * the stream it runs on, per phase: HG_PHASE_VERIFY = every launch of the
 * pairing-check kernel, HG_PHASE_AGGREGATE = the Combine fold of an aggregate
 * submission (plan, order, fold, finish), HG_PHASE_SUBMIT = a whole
 * verification submission (decode/aggregate + check). hg_timing_read_phase
 * returns (and clears) the summed time and the count of bracketed intervals;
 * hg_timing_read is hg_timing_read_phase(HG_PHASE_VERIFY). */
enum hg_phase { HG_PHASE_VERIFY = 0, HG_PHASE_AGGREGATE = 1, HG_PHASE_SUBMIT = 2, HG_NUM_PHASES = 3 };
int hg_timing_enable(hg_ctx* ctx, int on);
int hg_timing_read(hg_ctx* ctx, double* total_ms, int* launches);
int hg_timing_read_phase(hg_ctx* ctx, int phase, double* total_ms, int* launches);

/* Parity probe of the team Fp12 building blocks: elements are 384-byte GT
 * marshals. op: 0 a*b, 1 a^2, 2 cyclotomic a^2, 3 a^p, 4 a^(p^2), 5 a^-1,
 * 6 conj(a), 7 a^u, 8 final exponentiation, 9/10 table-program squarings. */
int hg_debug_fp12(hg_ctx* ctx, int op, const uint8_t* a, const uint8_t* b, size_t n, uint8_t* out);

/* Kernel probe of the GT path's signature side (bench.py per-kernel
 * roofline, the GPU suite's cross-kernel check): d_fe[r] (480 bytes, the
 * engine's internal GT layout) = FE(Miller(G2Base at -sig_r)) for the n
 * 64-byte signature marshals at d_sigs (context flavor), computed by kernel
 * 0: k_verify_sig padded (one wave per SIMD), 1: k_verify_sig unpadded,
 * 2: k_sig_scalars + k_sig_lines + k_verify_sig12 padded, 3: the same
 * unpadded (what a lane in flight runs: since r06 split into k_sig12_miller,
 * k_sig12_ninv, k_sig12_fe unless HG_SIG12_SPLIT=0), 4: k_verify_sig_split<2> (two
 * waves per check: the padded latency form for n <= 2048). Enqueued on `stream` (NULL: the
 * context's), ordered like every submission of the context. Replaces no
 * reference interface: the product paths choose the kernel themselves. */
int hg_sig_pairing_device(hg_ctx* ctx, const uint8_t* d_sigs, size_t n, uint8_t* d_fe, int kernel, void* stream);

/* Diagnostic builds only (-DHG_DIAG, tools/diag.py): per-block s_memtime
 * phase counters of the last pairing-check launch; HG_ERR_ARG otherwise. */
int hg_diag_read(hg_ctx* ctx, uint64_t* out, size_t n);

/* Wait for all work submitted on the context's stream. */
int hg_sync(hg_ctx* ctx);

/* Device memory held by the context (registry, its sums, GT tables,
 * workspaces), in bytes: the HBM one simul process's verifier costs. */
size_t hg_context_bytes(hg_ctx* ctx);

/* ---------------------------------------------------------------- packet intake
 * Handel.NewPacket's parse step for a batch of received packets (handel.go:
 * 127-152 -> validatePacket :371-385 -> parseSignatures :389-436): the origin
 * and level checks against the RECEIVING instance's partitioner
 * (partitioner.go:95-178), MultiSignature.Unmarshal of the wire bytes
 * (crypto.go:86-110: u16 BE blob length, the WilffBitSet blob = u16 BE bit
 * length + willf's u64 BE length and u64 BE words, then the signature
 * marshal), the bit-length and empty-bitset checks, and the optional
 * individual signature with its IndexAtLevel check. The output is the
 * verification requests processing.go's verifySignature runs on
 * (hg_verify_aggregate*), already in HBM for the device variant. */
typedef struct {
  int32_t origin;     /* Packet.Origin (net.go:36) */
  uint32_t receiver;  /* id of the Handel instance that received it (its partitioner) */
  uint32_t level;     /* Packet.Level (net.go:39; a byte on the wire) */
  uint32_t flags;     /* HG_PKT_HAS_IND: Packet.IndividualSig is non-nil */
  uint32_t ms_off, ms_len;   /* Packet.MultiSig = pool[ms_off .. ms_off + ms_len) */
  uint32_t ind_off, ind_len; /* Packet.IndividualSig = pool[ind_off .. ind_off + ind_len) */
} hg_packet;
#define HG_PKT_HAS_IND 1u
/* Words of bitset per request slot: ceil(largest level size / 64) for the
 * context's registry (the largest level holds 2^(ceil(log2 N) - 1) ids). */
size_t hg_packet_stride_words(hg_ctx* ctx);
/* Parses n packets against the context's registry size and flavor. Outputs
 * have 2n slots: slot i is packet i's multisignature, slot n + i its
 * individual signature as a one-bit multisignature of the level (handel.go:
 * 414-433). reqs[2n] (word_offset = slot * stride_words), words[2n *
 * stride_words] (bits at or above the bit length cleared), sigs[2n * 64] (the
 * signature marshal's first 64 bytes), codes[2n]: codes[i] = HG_OK or the
 * packet's first error in the reference's order; codes[n + i] = codes[i] if
 * that is an error, else HG_OK or HG_PKT_NO_IND. A packet whose individual
 * signature fails fails as a whole (parseSignatures returns the error and
 * NewPacket drops both). stride_words must be >= hg_packet_stride_words;
 * every pool range must lie inside pool_len (else HG_ERR_ARG). */
int hg_parse_packets(hg_ctx* ctx, const uint8_t* pool, size_t pool_len, const hg_packet* pkts, size_t n,
                     size_t stride_words, hg_request* reqs, uint64_t* words, uint8_t* sigs, int32_t* codes);
/* Device-resident variant (pool, pkts and every output on the device);
 * asynchronous on `stream`. A packet whose range leaves the pool gets
 * HG_ERR_ARG in its codes instead of a read outside it. */
int hg_parse_packets_device(hg_ctx* ctx, const uint8_t* d_pool, size_t pool_len, const hg_packet* d_pkts, size_t n,
                            size_t stride_words, hg_request* d_reqs, uint64_t* d_words, uint8_t* d_sigs,
                            int32_t* d_codes, void* stream);
/* The exact text the reference logs for packet p's code (with the level and
 * range values of the formatted errors), NUL-terminated into buf; returns the
 * full length (snprintf convention). */
int hg_packet_error(hg_ctx* ctx, int code, const hg_packet* p, char* buf, size_t cap);

/* ---------------------------------------------------------------- batcher
 * A launch-merging request queue on one context, for callers that verify one
 * multisignature at a time: each Handel instance's processLoop checks one
 * signature per step (processing.go:228-287 -> verifySignature :342-368) and
 * a simul process runs k instances concurrently (simul/node/main.go:63-131).
 * A dispatcher thread merges the queued requests into one
 * hg_verify_aggregate_msg batch (grouped by message, at most max_batch; an
 * idle dispatcher waits at most max_wait_us after the oldest request for
 * more) and hands every caller its own code. Verdicts are a pure function of
 * (msg, range, bitset, sig), so batching cannot change them. The context must
 * outlive the batcher. */
typedef struct hg_batcher hg_batcher;
typedef struct hg_ticket hg_ticket;
int hg_batcher_create(hg_ctx* ctx, size_t max_batch, unsigned max_wait_us, hg_batcher** out);
/* Verifies what is still queued, then stops the dispatcher. Tickets stay
 * valid: hg_batcher_wait on a ticket submitted before the destroy returns its
 * code even after the batcher is gone (a ticket holds its own state). */
void hg_batcher_destroy(hg_batcher* b);
/* Queues one request: req->offset / bitlen / level_size as in hg_request
 * (word_offset ignored), its ceil(bitlen/64) bitset words at `words`, the
 * 64-byte signature. Inputs are copied; the ticket is released by
 * hg_batcher_wait, exactly once. */
int hg_batcher_submit(hg_batcher* b, const uint8_t* msg, size_t len, const hg_request* req, const uint64_t* words,
                      const uint8_t* sig, hg_ticket** out);
/* Blocks until the ticket's batch ran; *code = its hg_code. Returns HG_OK, or
 * the batch's HG_ERR_ARG / HG_ERR_DEVICE. */
int hg_batcher_wait(hg_batcher* b, hg_ticket* t, int32_t* code);
/* hg_batcher_submit + hg_batcher_wait: one processing.go verifySignature. */
int hg_batcher_verify_aggregate(hg_batcher* b, const uint8_t* msg, size_t len, const hg_request* req,
                                const uint64_t* words, const uint8_t* sig, int32_t* code);
int hg_batcher_stats(hg_batcher* b, uint64_t* batches, uint64_t* requests);

/* ---------------------------------------------------------------- lanes
 * Several aggregate batches of one context in flight at once. A lane owns a
 * stream, device workspaces and pinned host staging; lanes share the
 * context's registry, hashed message and GT tables, which are read-only while
 * lanes run. A lane batch verifies against the context's CURRENT message
 * (hg_set_message / hg_prepare_aggregate_msg, called with every lane idle)
 * at the table level already built (hg_prepare_aggregate*): a lane never
 * builds tables. Used by the verifier service below; one thread per lane.
 * Lanes must be destroyed before their context. */
typedef struct hg_lane hg_lane;
/* max_batch requests and max_words bitset words per batch; overlap: the GT
 * fold beside the pairing kernel on a second stream of the lane. */
int hg_lane_create(hg_ctx* ctx, size_t max_batch, size_t max_words, int overlap, hg_lane** out);
void hg_lane_destroy(hg_lane* lane);
/* Pinned staging of the next batch: n requests (word_offset relative to
 * *words), their 64-byte signatures, nwords bitset words. The lane must be
 * idle. The pointers stay valid until the next hg_lane_stage. */
int hg_lane_stage(hg_lane* lane, size_t n, size_t nwords, hg_request** reqs, uint8_t** sigs, uint64_t** words);
/* Enqueues the staged batch (one host-to-device copy, the GT or G2 path,
 * the codes back to pinned memory); asynchronous. */
int hg_lane_submit(hg_lane* lane);
/* 1: the last batch is done (hg_lane_codes valid), 0: running, else an error code. */
int hg_lane_query(hg_lane* lane);
int hg_lane_wait(hg_lane* lane);
/* The last batch's n codes (pinned host memory, valid once it is done). */
const int32_t* hg_lane_codes(hg_lane* lane);
/* A batch already in HBM through the lane (the device twin of
 * hg_verify_aggregate_device_bits): enqueued on the lane's streams after the
 * caller's earlier work on `stream` (NULL: the context's stream), and `stream`
 * waits for the verdicts, so the caller reads d_codes / d_bits in its own
 * stream order while the next batch runs on another lane. d_bits may be NULL.
 * hg_lane_codes does not apply; hg_lane_query / hg_lane_wait do. */
int hg_lane_submit_device(hg_lane* lane, const hg_request* d_reqs, size_t n, const uint64_t* d_words,
                          const uint8_t* d_sigs, int32_t* d_codes, uint8_t* d_bits, void* stream);
/* 1 (the default): the lane's pairing kernel holds one wave per SIMD (the
 * lowest latency for one batch); 0: unpadded, so two batches in flight put
 * two pairing waves on a SIMD (throughput of a continuous stream). */
int hg_lane_set_pairing_padding(hg_lane* lane, int pad);
/* The latency form on a padded lane: its batches of at most max_checks
 * (<= 2048) checks run the pairing with each check's team over two waves
 * (k_verify_sig_split<2>: ~9 % shorter, twice the waves); 0 (the default,
 * or HG_SIG_W2_LANE_MAX): never. The verifier service sets it per batch while
 * the batches in flight leave a SIMD per wave. Takes effect at the next
 * submission. */
int hg_lane_set_latency_form(hg_lane* lane, int max_checks);
/* The lane's launch stream (a hipStream_t): passed as hg_lane_submit_device's
 * `stream`, the lane orders its batches only after its own earlier ones. */
void* hg_lane_stream(hg_lane* lane);
/* Builds the GT tables of the current message up to `level` (0..2, capped as
 * hg_prepare_aggregate caps) now; for owners of lanes that follow the volume
 * policy themselves. Synchronous. */
int hg_prepare_aggregate_level(hg_ctx* ctx, int level);

/* ---------------------------------------------------------------- verifier service
 * ONE process owns the GPU, the context, the registry and ONE set of GT
 * tables, and verifies the aggregate checks of many client processes that
 * reach it through a POSIX shared-memory object `name` (shm_open). Clients
 * use include/handel_client.h (libhandel_client.so: no GPU, no HIP runtime),
 * so simul's single-host layout — P OS processes of k Handel instances each
 * (simul/node/main.go:63-131), every instance's evaluator checking one
 * multisignature at a time (processing.go:228-287 -> verifySignature
 * :342-368) — shares one GPU without a HIP context per process. A dispatcher
 * thread merges queued requests into batches (grouped by message, at most
 * max_batch) and keeps up to `lanes` batches in flight (hg_lane_*); each
 * client learns its own verdicts. The context must outlive the service and
 * must not be used by others while it runs (the service switches its message
 * and builds its tables). */
typedef struct hg_service hg_service;
typedef struct {
  uint32_t slots;       /* request slots in the region (multiple of 64; default 8192) */
  uint32_t slot_bits;   /* largest bitset of one request (default: the registry size) */
  uint32_t channels;    /* client handles attached at once (default 256) */
  uint32_t lanes;       /* batches in flight on the GPU (default 8) */
  uint32_t max_batch;   /* requests per batch (default 4096) */
  uint32_t max_wait_us; /* a queued request waits at most this long for more to batch with (default 50) */
  uint32_t quiet_us;    /* ... or until no request has arrived for quiet_us (0 = off; the default) */
  int32_t prepare;      /* 1 (default): a message's first batch builds its top GT table level;
                           0: the context's volume policy (levels 1 and 2 after 16384 / 2^20 requests) */
  int32_t overlap;      /* 1 (default): the GT fold beside the pairing kernel inside each lane */
  int32_t follow;       /* 1 (default): ... or as soon as as many requests have arrived as finished
                           batches released (clients that submit their next check on a verdict:
                           the whole cohort is back), whichever comes first; 0: off */
} hg_service_config;
void hg_service_config_init(hg_service_config* cfg);
/* Creates the region (fails if `name` exists) and starts the dispatcher. */
int hg_service_create(hg_ctx* ctx, const char* name, const hg_service_config* cfg, hg_service** out);
/* The same protocol served by a CPU stand-in for the GPU (protocol tests
 * without a GPU): a request's code is HG_ERR_LEVEL if it fails the level
 * check against an nreg-key registry, 77 if its bitset words do not match
 * sig[1..8] (the xor of the words, little-endian), else HG_ERR_SIG_INVALID
 * if sig[0] == 1, else HG_OK; each batch completes delay_us after launch. */
int hg_service_create_echo(const char* name, const hg_service_config* cfg, uint32_t nreg, uint32_t delay_us,
                           hg_service** out);
/* Verifies what is queued, stops the dispatcher, wakes every client and
 * removes the region's name. */
void hg_service_destroy(hg_service* svc);
/* batches launched, requests verified, most batches in flight at once */
int hg_service_stats(hg_service* svc, uint64_t* batches, uint64_t* requests, uint64_t* max_in_flight);

#ifdef __cplusplus
}
#endif
#endif /* HANDEL_GPU_H */
