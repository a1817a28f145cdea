// Package hip is the Go side of the drop-in boundary: Handel's bn256 plugin
// (the Constructor / PublicKey / SigBLS / SecretKey types of
// bn256/go/bn256.go:34-204 and bn256/cf/bn256.go) backed by the MI355X
// engine through its C ABI (include/handel_gpu.h of this repository).
//
// It is source for a maintainer to drop into the Handel tree at bn256/hip;
// Go is not installed where this repository is built, so nothing here has
// been compiled. Build flags come from the environment (INTEGRATION.md):
//
//	export CGO_CFLAGS="-I$HANDEL_AMD/include"
//	export CGO_LDFLAGS="-L$HANDEL_AMD/handel_amd/_build -Wl,-rpath,$HANDEL_AMD/handel_amd/_build"
//
// The C library copies every input into device memory before it returns, so
// the cgo pointer rules hold: C never keeps a Go pointer.
package hip

/*
#cgo LDFLAGS: -lhandel_gpu
#include <stdlib.h>
#include "handel_gpu.h"
*/
import "C"

import (
	"errors"
	"fmt"
	"math"
	"sync"
	"unsafe"
)

// Flavor selects which upstream library's Unmarshal rules the engine mirrors
// (simul/lib/config.go:211-225 maps "bn256" and "bn256/cf" to cloudflare,
// "bn256/go" to golang.org/x/crypto).
type Flavor int

const (
	// FlavorGo mirrors golang.org/x/crypto/bn256 (package bn256/go).
	FlavorGo Flavor = C.HG_FLAVOR_GO
	// FlavorCF mirrors github.com/cloudflare/bn256 (package bn256/cf).
	FlavorCF Flavor = C.HG_FLAVOR_CF
)

// Per-request result codes of the C ABI (enum hg_code).
const (
	codeOK         = C.HG_OK
	codeSigInvalid = C.HG_ERR_SIG_INVALID
	codeHashEOF    = C.HG_ERR_HASH_EOF
	codeLevel      = C.HG_ERR_LEVEL
	codeEmptyAgg   = C.HG_ERR_EMPTY_AGG
)

// DeviceError is returned when a whole submission fails (HG_ERR_ARG or
// HG_ERR_DEVICE): no request of that submission has a verdict, and callers
// must treat every one of them as unverified (fail closed).
type DeviceError struct {
	Code int
	Msg  string
}

func (e *DeviceError) Error() string {
	return fmt.Sprintf("hip: engine call failed (code %d): %s", e.Code, e.Msg)
}

// Engine owns one device context: the decoded registry, the hashed message
// cache and the G2Base line table. Every method is safe for concurrent use
// (the C library serialises submitters on the context).
type Engine struct {
	ctx    *C.hg_ctx
	flavor Flavor
	once   sync.Once
	// registry bookkeeping for index lookups (see registry.go)
	regMu sync.RWMutex
	reg   *Registry
	// VerifySignature batcher (batcher.go), started on first use
	bOnce sync.Once
	b     *batcher
}

// NewEngine opens device `device` (a HIP ordinal) with the Unmarshal rules
// of `flavor`.
func NewEngine(device int, flavor Flavor) (*Engine, error) {
	e := &Engine{flavor: flavor}
	if rc := C.hg_create(C.int(device), C.int(flavor), &e.ctx); rc != C.HG_OK {
		return nil, &DeviceError{Code: int(rc), Msg: "hg_create failed"}
	}
	return e, nil
}

// Close stops the batcher and releases the device context. No call may be in
// flight or follow it.
func (e *Engine) Close() {
	e.once.Do(func() {
		if e.b != nil {
			e.b.close()
		}
		C.hg_destroy(e.ctx)
		e.ctx = nil
	})
}

// Flavor returns the Unmarshal rules this engine mirrors.
func (e *Engine) Flavor() Flavor { return e.flavor }

func (e *Engine) fail(rc C.int) error {
	return &DeviceError{Code: int(rc), Msg: C.GoString(C.hg_last_error(e.ctx))}
}

// CodeError is the error the reference returns for a per-request code, as
// PublicKey.VerifySignature / UnmarshalBinary return it (nil for HG_OK).
func (e *Engine) CodeError(code int32) error {
	if code == codeOK {
		return nil
	}
	return errors.New(C.GoString(C.hg_code_string(C.int(code), C.int(e.flavor))))
}

// ProcessingError is the error processing.go's verifySignature returns for a
// per-request code (processing.go:342-368): VerifySignature's errors wrapped
// as "handel: <err>", the level check's own text unwrapped.
func (e *Engine) ProcessingError(code int32) error {
	if code == codeOK {
		return nil
	}
	return errors.New(C.GoString(C.hg_processing_error_string(C.int(code), C.int(e.flavor))))
}

// bytePtr / wordPtr / codePtr guard empty slices: the C ABI takes NULL with a
// zero length, and &s[0] on an empty slice panics.
func bytePtr(b []byte) *C.uint8_t {
	if len(b) == 0 {
		return nil
	}
	return (*C.uint8_t)(unsafe.Pointer(&b[0]))
}

func wordPtr(w []uint64) *C.uint64_t {
	if len(w) == 0 {
		return nil
	}
	return (*C.uint64_t)(unsafe.Pointer(&w[0]))
}

func codePtr(c []int32) *C.int32_t {
	if len(c) == 0 {
		return nil
	}
	return (*C.int32_t)(unsafe.Pointer(&c[0]))
}

// failedCodes pre-fills a code array with a non-OK value, so a submission
// that returns early can never read as "every signature valid".
func failedCodes(n int) []int32 {
	c := make([]int32, n)
	for i := range c {
		c[i] = C.HG_ERR_DEVICE
	}
	return c
}

// SetMessage hashes msg to G1 once (hashedMessage, bn256/go/bn256.go:210-218)
// and caches it on the device. It returns the hash error ("EOF") when the
// digest is not a valid scalar; checks then fail with that error.
func (e *Engine) SetMessage(msg []byte) error {
	rc := C.hg_set_message(e.ctx, bytePtr(msg), C.size_t(len(msg)))
	switch rc {
	case C.HG_OK:
		return nil
	case C.HG_ERR_HASH_EOF:
		return e.CodeError(codeHashEOF)
	}
	return e.fail(rc)
}

// PrepareAggregate makes msg the context's message and builds the tables of
// aggregate verification for it and the loaded registry now (e(H, pk_i) and
// the GT window/block products: ≈ 15 ms for 4000 keys) instead of in the
// first aggregate call. Call it once per Handel run after LoadRegistry.
// Without it the engine builds the tables by request volume (see
// AggregateTables).
func (e *Engine) PrepareAggregate(msg []byte) error {
	// hashing and the build under one lock hold of the context
	// (hg_prepare_aggregate_msg): a concurrent caller with another message
	// cannot take the tables in between
	switch rc := C.hg_prepare_aggregate_msg(e.ctx, bytePtr(msg), C.size_t(len(msg))); rc {
	case C.HG_OK:
		return nil
	case C.HG_ERR_HASH_EOF:
		return e.CodeError(codeHashEOF)
	default:
		return e.fail(rc)
	}
}

// AggregateTables reports the table level aggregate checks run at: 0 = G2
// key fold + two pairings (a message's first 16384 requests), 1 = GT fold over
// 8-key windows, 2 = over 16-key windows (after PrepareAggregate, or 2^20
// requests).
func (e *Engine) AggregateTables() int {
	return int(C.hg_aggregate_tables(e.ctx))
}

// SetAggregateLevel pins the table level of aggregate checks (0..2) or, with
// -1, returns them to the volume policy (hg_set_aggregate_level).
func (e *Engine) SetAggregateLevel(level int) error {
	if rc := C.hg_set_aggregate_level(e.ctx, C.int(level)); rc != C.HG_OK {
		return e.fail(rc)
	}
	return nil
}

// SetTableBudget bounds the HBM of this engine's aggregate tables: processes
// sharing one GPU (simul's P processes x k instances) each take a share. A
// level that does not fit is skipped (hg_set_table_budget).
func (e *Engine) SetTableBudget(bytes uint64) error {
	if rc := C.hg_set_table_budget(e.ctx, C.size_t(bytes)); rc != C.HG_OK {
		return e.fail(rc)
	}
	return nil
}

// SetVerifySplit selects config 2's form for this engine: true runs
// VerifyBatch as the split form (the Miller loop on a compact team region,
// then the 12-lane final exponentiation), the faster one when several engines
// each keep a batch in flight on one GPU; same verdicts (hg_set_verify_split).
func (e *Engine) SetVerifySplit(on bool) error {
	v := C.int(0)
	if on {
		v = 1
	}
	if rc := C.hg_set_verify_split(e.ctx, v); rc != C.HG_OK {
		return e.fail(rc)
	}
	return nil
}

// RegistryNonG2 is the number of loaded registry keys on the twist but
// outside G2 (accepted by x/crypto's Unmarshal); such a registry is checked
// with the G2 point fold and two pairings (hg_registry_non_g2).
func (e *Engine) RegistryNonG2() int { return int(C.hg_registry_non_g2(e.ctx)) }

// DeviceBytes is the device memory the context holds (hg_context_bytes).
func (e *Engine) DeviceBytes() uint64 { return uint64(C.hg_context_bytes(e.ctx)) }

// VerifyBatch runs n = len(sigs)/64 independent PublicKey.VerifySignature(msg,
// sig) checks (bn256/go/bn256.go:82-94) in one launch; pks holds n 128-byte
// key marshals. Hashing and checking happen under one lock hold of the
// context, so callers with different messages cannot interleave.
func (e *Engine) VerifyBatch(msg, pks, sigs []byte) ([]int32, error) {
	n := len(sigs) / 64
	if len(sigs) != 64*n || len(pks) != 128*n {
		return nil, &DeviceError{Code: C.HG_ERR_ARG, Msg: "VerifyBatch: pks/sigs sizes"}
	}
	codes := failedCodes(n)
	rc := C.hg_verify_batch_msg(e.ctx, bytePtr(msg), C.size_t(len(msg)), bytePtr(pks), bytePtr(sigs), C.size_t(n),
		codePtr(codes))
	if rc != C.HG_OK {
		return nil, e.fail(rc)
	}
	return codes, nil
}

// Request is one aggregate check (processing.go:342-368 verifySignature):
// the level's registry range starts at Offset and has LevelSize keys; Words
// holds the bitset (willf layout: bit i = Words[i>>6] bit i&63) of BitLen
// bits; Sig is the 64-byte aggregate signature marshal.
type Request struct {
	Offset    int
	LevelSize int
	BitLen    int
	Words     []uint64
	Sig       []byte
}

type packed struct {
	reqs  []C.hg_request
	words []uint64
	sigs  []byte
}

func pack(reqs []Request) (*packed, error) {
	p := &packed{reqs: make([]C.hg_request, len(reqs)), sigs: make([]byte, 64*len(reqs))}
	nw := 0
	for _, r := range reqs {
		nw += len(r.Words)
	}
	p.words = make([]uint64, 0, nw)
	for i, r := range reqs {
		if r.Offset < 0 || r.LevelSize < 0 || r.BitLen < 0 || len(r.Words) < (r.BitLen+63)/64 {
			return nil, &DeviceError{Code: C.HG_ERR_ARG, Msg: fmt.Sprintf("request %d: malformed range or bitset", i)}
		}
		p.reqs[i] = C.hg_request{
			offset:      C.uint32_t(r.Offset),
			bitlen:      C.uint32_t(r.BitLen),
			level_size:  C.uint32_t(r.LevelSize),
			word_offset: C.uint32_t(len(p.words)),
		}
		p.words = append(p.words, r.Words[:(r.BitLen+63)/64]...)
		// a wrong-length signature cannot decode: zero bytes then decode as
		// infinity in x/crypto, so a short signature is refused here instead
		if len(r.Sig) != 64 {
			return nil, &DeviceError{Code: C.HG_ERR_ARG, Msg: fmt.Sprintf("request %d: signature is %d bytes", i, len(r.Sig))}
		}
		copy(p.sigs[64*i:], r.Sig)
	}
	return p, nil
}

// VerifyAggregate runs the batched verifySignature: for every request the
// Combine fold over the set bits of its level range, then VerifySignature on
// msg. It returns one code per request (hg_code) and, when wantKeys, the
// 128-byte marshal of every aggregate key.
func (e *Engine) VerifyAggregate(msg []byte, reqs []Request, wantKeys bool) ([]int32, []byte, error) {
	p, err := pack(reqs)
	if err != nil {
		return nil, nil, err
	}
	codes := failedCodes(len(reqs))
	var agg []byte
	if wantKeys {
		agg = make([]byte, 128*len(reqs))
	}
	var reqPtr *C.hg_request
	if len(p.reqs) > 0 {
		reqPtr = &p.reqs[0]
	}
	rc := C.hg_verify_aggregate_msg(e.ctx, bytePtr(msg), C.size_t(len(msg)), reqPtr, C.size_t(len(reqs)),
		wordPtr(p.words), C.size_t(len(p.words)), bytePtr(p.sigs), codePtr(codes), bytePtr(agg))
	if rc != C.HG_OK {
		return nil, nil, e.fail(rc)
	}
	return codes, agg, nil
}

// AggregateKeys is the Combine fold alone: the marshalled aggregate public
// key of every request (codes: HG_OK, HG_ERR_LEVEL or HG_ERR_EMPTY_AGG).
func (e *Engine) AggregateKeys(reqs []Request) ([]byte, []int32, error) {
	for i := range reqs {
		if reqs[i].Sig == nil {
			reqs[i].Sig = make([]byte, 64)
		}
	}
	p, err := pack(reqs)
	if err != nil {
		return nil, nil, err
	}
	codes := failedCodes(len(reqs))
	out := make([]byte, 128*len(reqs))
	var reqPtr *C.hg_request
	if len(p.reqs) > 0 {
		reqPtr = &p.reqs[0]
	}
	rc := C.hg_aggregate_pk(e.ctx, reqPtr, C.size_t(len(reqs)), wordPtr(p.words), C.size_t(len(p.words)),
		bytePtr(out), codePtr(codes))
	if rc != C.HG_OK {
		return nil, nil, e.fail(rc)
	}
	return out, codes, nil
}

// VerifyMultiSignatures is crypto.go:120-137 VerifyMultiSignature for every
// (bitset, signature) pair: bitLens[i] must equal the registry size, or the
// request fails with "verify multisignature: inconsistent sizes". It runs as
// full-range aggregate requests under one lock hold with the message (the C
// ABI's hg_verify_multisig is the same check without the message).
func (e *Engine) VerifyMultiSignatures(msg []byte, bitLens []int, words [][]uint64, sigs []byte) ([]int32, error) {
	n := len(bitLens)
	if len(words) != n || len(sigs) != 64*n {
		return nil, &DeviceError{Code: C.HG_ERR_ARG, Msg: "VerifyMultiSignatures: sizes"}
	}
	size := int(C.hg_registry_size(e.ctx))
	reqs := make([]Request, n)
	for i := range reqs {
		reqs[i] = Request{Offset: 0, LevelSize: size, BitLen: bitLens[i], Words: words[i], Sig: sigs[64*i : 64*i+64]}
		if bitLens[i] != size {
			// fails the range check on the device; the code is replaced below
			reqs[i].BitLen, reqs[i].Words = 0, nil
		}
	}
	codes, _, err := e.VerifyAggregate(msg, reqs, false)
	if err != nil {
		return nil, err
	}
	for i := range codes {
		if bitLens[i] != size {
			codes[i] = C.HG_ERR_MULTI_SIZES
		}
	}
	return codes, nil
}

// CombineG1 is SigBLS.Combine batched: out[i] = a[i] + b[i] (64-byte marshals).
func (e *Engine) CombineG1(a, b []byte) ([]byte, []int32, error) {
	n := len(a) / 64
	if len(a) != 64*n || len(b) != len(a) {
		return nil, nil, &DeviceError{Code: C.HG_ERR_ARG, Msg: "CombineG1: sizes"}
	}
	out := make([]byte, len(a))
	codes := failedCodes(n)
	if rc := C.hg_combine_g1(e.ctx, bytePtr(a), bytePtr(b), C.size_t(n), bytePtr(out), codePtr(codes)); rc != C.HG_OK {
		return nil, nil, e.fail(rc)
	}
	return out, codes, nil
}

// CombineG2 is PublicKey.Combine batched: out[i] = a[i] + b[i] (128-byte marshals).
func (e *Engine) CombineG2(a, b []byte) ([]byte, []int32, error) {
	n := len(a) / 128
	if len(a) != 128*n || len(b) != len(a) {
		return nil, nil, &DeviceError{Code: C.HG_ERR_ARG, Msg: "CombineG2: sizes"}
	}
	out := make([]byte, len(a))
	codes := failedCodes(n)
	if rc := C.hg_combine_g2(e.ctx, bytePtr(a), bytePtr(b), C.size_t(n), bytePtr(out), codePtr(codes)); rc != C.HG_OK {
		return nil, nil, e.fail(rc)
	}
	return out, codes, nil
}

// Keygen computes pk = k*G2 (NewKeyPair, bn256/go/bn256.go:129-142) for
// 32-byte big-endian scalars.
func (e *Engine) Keygen(scalars []byte) ([]byte, error) {
	n := len(scalars) / 32
	if len(scalars) != 32*n {
		return nil, &DeviceError{Code: C.HG_ERR_ARG, Msg: "Keygen: scalars must be 32 bytes each"}
	}
	out := make([]byte, 128*n)
	if rc := C.hg_keygen(e.ctx, bytePtr(scalars), C.size_t(n), bytePtr(out)); rc != C.HG_OK {
		return nil, e.fail(rc)
	}
	return out, nil
}

// Sign computes sig = k*H(msg) (SecretKey.Sign, bn256/go/bn256.go:146-154)
// for 32-byte big-endian scalars; the hash error comes back as "EOF".
func (e *Engine) Sign(msg, scalars []byte) ([]byte, error) {
	n := len(scalars) / 32
	if len(scalars) != 32*n {
		return nil, &DeviceError{Code: C.HG_ERR_ARG, Msg: "Sign: scalars must be 32 bytes each"}
	}
	out := make([]byte, 64*n)
	rc := C.hg_sign_msg(e.ctx, bytePtr(msg), C.size_t(len(msg)), bytePtr(scalars), C.size_t(n), bytePtr(out))
	switch rc {
	case C.HG_OK:
		return out, nil
	case C.HG_ERR_HASH_EOF:
		return nil, e.CodeError(codeHashEOF)
	}
	return nil, e.fail(rc)
}

// loadRegistry uploads n = len(pks)/128 key marshals and builds the window
// and block tables the aggregate fold uses. On failure the context holds no
// registry; codes[i] is the decode code of key i.
func (e *Engine) loadRegistry(pks []byte) ([]int32, error) {
	n := len(pks) / 128
	codes := failedCodes(n)
	rc := C.hg_registry_load(e.ctx, bytePtr(pks), C.size_t(n), codePtr(codes))
	if rc == C.HG_ERR_PK_UNMARSHAL {
		for i, c := range codes {
			if c != codeOK {
				return codes, fmt.Errorf("registry key %d: %v", i, e.CodeError(c))
			}
		}
	}
	if rc != C.HG_OK {
		return codes, e.fail(rc)
	}
	return codes, nil
}

// Packet mirrors handel.Packet (net.go:34-44) field for field, so a caller
// converts with hip.Packet(*p).
type Packet struct {
	Origin        int32
	Level         byte
	MultiSig      []byte
	IndividualSig []byte
}

// ParsedPacket is Handel.NewPacket's parse step for one packet (handel.go:
// 127-152): Err is what validatePacket / parseSignatures return (nil when the
// packet is accepted); MultiSig is the verifySignature request of the
// multisignature, Individual the individual signature as a one-bit request of
// the level (nil when the packet carried none).
type ParsedPacket struct {
	Err        error
	MultiSig   Request
	Individual *Request
}

// ParsePackets parses a batch of packets received by the instances
// receivers[i] (hg_parse_packets: origin and level checks, MultiSignature /
// WilffBitSet / willf unmarshal, bit length, empty set, individual signature
// and IndexAtLevel, in the reference's order).
func (e *Engine) ParsePackets(receivers []int, pkts []Packet) ([]ParsedPacket, error) {
	n := len(pkts)
	if len(receivers) != n {
		return nil, &DeviceError{Code: C.HG_ERR_ARG, Msg: "ParsePackets: one receiver per packet"}
	}
	if n == 0 {
		return nil, nil
	}
	var pool []byte
	recs := make([]C.hg_packet, n)
	for i, p := range pkts {
		// pool offsets and lengths are 32-bit in hg_packet: a batch whose pool
		// would pass 4 GiB is refused instead of wrapping into wrong bytes
		if uint64(len(pool))+uint64(len(p.MultiSig))+uint64(len(p.IndividualSig)) > math.MaxUint32 {
			return nil, &DeviceError{Code: C.HG_ERR_ARG, Msg: "ParsePackets: the batch's packets exceed 4 GiB; split it"}
		}
		recs[i] = C.hg_packet{origin: C.int32_t(p.Origin), receiver: C.uint32_t(receivers[i]),
			level: C.uint32_t(p.Level), ms_off: C.uint32_t(len(pool)), ms_len: C.uint32_t(len(p.MultiSig))}
		pool = append(pool, p.MultiSig...)
		if p.IndividualSig != nil {
			recs[i].flags = C.HG_PKT_HAS_IND
			recs[i].ind_off, recs[i].ind_len = C.uint32_t(len(pool)), C.uint32_t(len(p.IndividualSig))
			pool = append(pool, p.IndividualSig...)
		}
	}
	stride := int(C.hg_packet_stride_words(e.ctx))
	reqs := make([]C.hg_request, 2*n)
	words := make([]uint64, 2*n*stride)
	sigs := make([]byte, 2*n*64)
	codes := failedCodes(2 * n)
	rc := C.hg_parse_packets(e.ctx, bytePtr(pool), C.size_t(len(pool)), &recs[0], C.size_t(n), C.size_t(stride),
		&reqs[0], wordPtr(words), bytePtr(sigs), codePtr(codes))
	if rc != C.HG_OK {
		return nil, e.fail(rc)
	}
	slot := func(k int) Request {
		r := reqs[k]
		nw := (int(r.bitlen) + 63) / 64
		w := make([]uint64, nw)
		copy(w, words[int(r.word_offset):int(r.word_offset)+nw])
		s := make([]byte, 64)
		copy(s, sigs[64*k:64*k+64])
		return Request{Offset: int(r.offset), LevelSize: int(r.level_size), BitLen: int(r.bitlen), Words: w, Sig: s}
	}
	out := make([]ParsedPacket, n)
	buf := make([]byte, 256)
	for i := range out {
		if codes[i] != C.HG_OK {
			C.hg_packet_error(e.ctx, C.int(codes[i]), &recs[i], (*C.char)(unsafe.Pointer(&buf[0])), C.size_t(len(buf)))
			out[i].Err = errors.New(C.GoString((*C.char)(unsafe.Pointer(&buf[0]))))
			continue
		}
		out[i].MultiSig = slot(i)
		if codes[n+i] == C.HG_OK {
			ind := slot(n + i)
			out[i].Individual = &ind
		}
	}
	return out, nil
}
