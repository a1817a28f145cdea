// Package hipsvc submits Handel's signature checks to the GPU-owning verifier
// process (hg_verifierd; hg_service_* in include/handel_gpu.h) through shared
// memory, with cgo bindings of include/handel_client.h. The library it links,
// libhandel_client.so, has no GPU or HIP dependency: a simul node process
// (simul/node/main.go:63-131: k Handel instances per process) uses it instead
// of opening a GPU context of its own, so P processes share one GPU, one
// registry and one set of GT tables.
//
// Go is not installed where this was written: this file has not been
// compiled. The C calls it makes are exercised from C
// (tests/native/handel_proxy.c -D 1) and Python (handel_amd/service.py).
package hipsvc

/*
#cgo LDFLAGS: -lhandel_client
#include <stdlib.h>
#include "handel_client.h"
*/
import "C"

import (
	"errors"
	"fmt"
	"sync"
	"unsafe"

	"github.com/ConsenSys/handel"
)

// Request is one verifySignature (processing.go:342-368): the level's
// registry range [Offset, Offset + LevelSize), the bitset of BitLen bits as
// willf words (bit i = Words[i >> 6] bit i & 63), the 64-byte signature.
type Request struct {
	Offset, LevelSize, BitLen int
	Words                     []uint64
	Sig                       []byte
}

// Client is one handle on the verifier's region: a completion channel polled
// by one goroutine (one OS thread parked in hg_client_wait_any), which hands
// each code to the goroutine waiting for it. Verify may be called from any
// number of goroutines (k Handel instances).
type Client struct {
	h       *C.hg_client
	mu      sync.Mutex
	waiting map[uint64]chan int32
	early   map[uint64]int32 // codes collected before their waiter registered
	done    chan struct{}    // closed by Close: poll returns
	polled  chan struct{}    // closed by poll when it returns
	dead    error
	// hmu guards the handle itself: submits hold it shared, Close exclusively,
	// so hg_client_close never runs while a C call uses the handle
	hmu       sync.RWMutex
	closed    bool
	closeOnce sync.Once
	texts     map[int32]string // code -> processing.go error text (read-only after Open)
}

var errClosed = errors.New("hipsvc: client closed")

// Open attaches to the verifier region `name` (hg_verifierd --name).
func Open(name string) (*Client, error) {
	cn := C.CString(name)
	defer C.free(unsafe.Pointer(cn))
	var h *C.hg_client
	if rc := C.hg_client_open(cn, &h); rc != C.HG_OK {
		return nil, fmt.Errorf("hipsvc: cannot attach to %s (code %d)", name, int(rc))
	}
	c := &Client{h: h, waiting: map[uint64]chan int32{}, early: map[uint64]int32{}, done: make(chan struct{}),
		polled: make(chan struct{}), texts: map[int32]string{}}
	// every code's text, taken while the handle is certainly open: a verdict
	// delivered as Close runs keeps its own error (handel_gpu.h hg_code values
	// 0..29, 100, 101; anything else maps to "device error")
	for code := int32(0); code <= 101; code++ {
		c.texts[code] = C.GoString(C.hg_client_processing_error_string(h, C.int(code)))
	}
	go c.poll()
	return c, nil
}

// poll collects finished tickets and delivers their codes.
func (c *Client) poll() {
	defer close(c.polled)
	tickets := make([]C.uint64_t, 512)
	codes := make([]C.int32_t, 512)
	for {
		n := C.hg_client_wait_any(c.h, &tickets[0], &codes[0], C.size_t(len(tickets)), 100000)
		select {
		case <-c.done:
			return
		default:
		}
		if n < 0 {
			c.failAll(errors.New("hipsvc: the verifier stopped"))
			return
		}
		c.mu.Lock()
		for i := 0; i < int(n); i++ {
			t := uint64(tickets[i])
			if ch, ok := c.waiting[t]; ok {
				ch <- int32(codes[i])
				delete(c.waiting, t)
			} else {
				c.early[t] = int32(codes[i])
			}
		}
		c.mu.Unlock()
	}
}

// failAll ends every registered waiter with err (they return it).
func (c *Client) failAll(err error) {
	c.mu.Lock()
	if c.dead == nil {
		c.dead = err
	}
	for t, ch := range c.waiting {
		ch <- -1
		delete(c.waiting, t)
	}
	c.mu.Unlock()
}

// Close detaches (tickets in flight are dropped; their Verify calls return
// an error). The poll goroutine is stopped first — it may sit in
// hg_client_wait_any for up to 100 ms — and no submit is in progress when
// the handle is released (handel_client.h: close must not run concurrently
// with the handle's other calls). Safe to call more than once.
func (c *Client) Close() {
	c.closeOnce.Do(func() {
		close(c.done)
		<-c.polled
		c.failAll(errClosed)
		c.hmu.Lock()
		c.closed = true
		C.hg_client_close(c.h)
		c.h = nil
		c.hmu.Unlock()
	})
}

func u8ptr(b []byte) *C.uint8_t {
	if len(b) == 0 {
		return nil
	}
	return (*C.uint8_t)(unsafe.Pointer(&b[0]))
}

// Verify is one processing.go verifySignature: nil, or the error the
// reference returns ("handel: inconsistent bitset with given level",
// "handel: bn256: signature invalid", "handel: EOF", ...).
func (c *Client) Verify(msg []byte, r Request) error {
	if len(r.Sig) != 64 {
		return errors.New("bn256: multisig can't unmarshal")
	}
	if len(r.Words) < (r.BitLen+63)/64 {
		return errors.New("hipsvc: fewer bitset words than bits")
	}
	req := C.hg_request{offset: C.uint32_t(r.Offset), bitlen: C.uint32_t(r.BitLen),
		level_size: C.uint32_t(r.LevelSize)}
	var words *C.uint64_t
	if len(r.Words) > 0 {
		words = (*C.uint64_t)(unsafe.Pointer(&r.Words[0]))
	}
	var t C.uint64_t
	c.hmu.RLock()
	if c.closed {
		c.hmu.RUnlock()
		return errClosed
	}
	// the library copies every input before returning (cgo pointer rules hold)
	rc := C.hg_client_submit(c.h, u8ptr(msg), C.size_t(len(msg)), &req, words, u8ptr(r.Sig), &t)
	c.hmu.RUnlock()
	if rc != C.HG_OK {
		return fmt.Errorf("hipsvc: submit refused (code %d)", int(rc))
	}
	ch := make(chan int32, 1)
	c.mu.Lock()
	if c.dead != nil {
		c.mu.Unlock()
		return c.dead
	}
	if code, ok := c.early[uint64(t)]; ok {
		delete(c.early, uint64(t))
		c.mu.Unlock()
		return c.codeError(code)
	}
	c.waiting[uint64(t)] = ch
	c.mu.Unlock()
	code := <-ch
	if code < 0 {
		c.mu.Lock()
		err := c.dead
		c.mu.Unlock()
		return err
	}
	return c.codeError(code)
}

// codeError maps an hg_code to processing.go's error (nil for HG_OK), from
// the table Open took (hg_client_processing_error_string depends only on the
// flavor), so it never needs the handle: a real verdict that arrives while
// Close runs stays that verdict, not errClosed.
func (c *Client) codeError(code int32) error {
	if code == C.HG_OK {
		return nil
	}
	if t, ok := c.texts[code]; ok {
		return errors.New(t)
	}
	return errors.New("device error")
}

// Verifier is a handel.BatchVerifier (go/handel/batched_processing.go) over
// the service for a registry of n identities whose IDs are their indices (the
// simul registry): each request's level range is its identities' ID range.
func (c *Client) Verifier(n int) handel.BatchVerifier { return &verifier{c: c, n: n} }

type verifier struct {
	c *Client
	n int
}

func (v *verifier) VerifyBatch(msg []byte, reqs []handel.BatchRequest) []error {
	out := make([]error, len(reqs))
	var wg sync.WaitGroup
	for i, q := range reqs {
		off := 0
		if len(q.Identities) > 0 {
			off = int(q.Identities[0].ID())
			for j, id := range q.Identities {
				if int(id.ID()) != off+j || off+len(q.Identities) > v.n {
					out[i] = errors.New("hipsvc: level identities are not a contiguous registry range")
					break
				}
			}
		}
		if out[i] != nil {
			continue
		}
		sig, err := q.MultiSig.Signature.MarshalBinary()
		if err != nil {
			out[i] = err
			continue
		}
		bs := q.MultiSig.BitSet
		n := bs.BitLength()
		words := make([]uint64, (n+63)/64)
		for b, ok := bs.NextSet(0); ok && b < n; b, ok = bs.NextSet(b + 1) {
			words[b>>6] |= 1 << uint(b&63)
		}
		wg.Add(1)
		go func(i int, r Request) { // every request in flight at once: one service batch
			defer wg.Done()
			out[i] = v.c.Verify(msg, r)
		}(i, Request{Offset: off, LevelSize: len(q.Identities), BitLen: n, Words: words, Sig: sig})
	}
	wg.Wait()
	return out
}
