package hip

import (
	"crypto/rand"
	"crypto/sha256"
	"encoding/hex"
	"errors"
	"io"
	"math/big"
	"os"
	"strconv"
	"sync"

	"github.com/ConsenSys/handel"
)

// Order is the order n of G1, G2 and GT (the scalar field of the keys).
var Order, _ = new(big.Int).SetString(
	"65000549695646603732796438742359905742570406053903786389881062969044166799969", 10)

var (
	defaultMu     sync.Mutex
	defaultEngine = map[Flavor]*Engine{}
)

// Default returns the process-wide engine for flavor (device from HG_DEVICE,
// default 0) — the counterpart of bn256/go's package-level state (G2Base,
// Hash). k Handel instances in one process share it, and their concurrent
// VerifySignature calls are merged into one launch by the engine's batcher.
func Default(flavor Flavor) (*Engine, error) {
	defaultMu.Lock()
	defer defaultMu.Unlock()
	if e, ok := defaultEngine[flavor]; ok {
		return e, nil
	}
	dev := 0
	if s := os.Getenv("HG_DEVICE"); s != "" {
		d, err := strconv.Atoi(s)
		if err != nil {
			return nil, err
		}
		dev = d
	}
	e, err := NewEngine(dev, flavor)
	if err != nil {
		return nil, err
	}
	defaultEngine[flavor] = e
	return e, nil
}

func mustDefault(flavor Flavor) *Engine {
	e, err := Default(flavor)
	if err != nil {
		// there is no CPU path: without the device the plugin cannot work
		panic(err)
	}
	return e
}

// Constructor implements handel.Constructor and the simul/lib extension
// (bn256/go/bn256.go:34-67; simul/lib/crypto.go:18-50).
type Constructor struct {
	e *Engine
}

// NewConstructor returns a Constructor on the default engine with
// golang.org/x/crypto's Unmarshal rules (bn256/go/bn256.go:40-42).
func NewConstructor() *Constructor {
	return &Constructor{e: mustDefault(FlavorGo)}
}

// NewConstructorCF is NewConstructor with cloudflare/bn256's Unmarshal
// rules (bn256/cf: the curve "bn256" of every shipped simulation config).
func NewConstructorCF() *Constructor {
	return &Constructor{e: mustDefault(FlavorCF)}
}

// NewConstructorOn binds a Constructor to an explicit engine.
func NewConstructorOn(e *Engine) *Constructor { return &Constructor{e: e} }

// Engine returns the engine the constructor's objects use.
func (c *Constructor) Engine() *Engine { return c.e }

// Signature implements handel.Constructor.
func (c *Constructor) Signature() handel.Signature { return &SigBLS{e: c.e} }

// PublicKey implements handel.Constructor: the empty key, identity of Combine.
func (c *Constructor) PublicKey() handel.PublicKey { return &PublicKey{e: c.e} }

// SecretKey implements the simul/lib Constructor interface.
func (c *Constructor) SecretKey() handel.SecretKey { return &SecretKey{e: c.e} }

// KeyPair implements the simul/lib Constructor interface (panics on a reader
// error, as bn256/go/bn256.go:60-67 does).
func (c *Constructor) KeyPair(r io.Reader) (handel.SecretKey, handel.PublicKey) {
	sk, pk, err := newKeyPair(c.e, r)
	if err != nil {
		panic(err)
	}
	return sk, pk
}

// PublicKey is a G2 point (bn256/go/bn256.go:69-121) in one of three forms:
//   - empty (the Constructor's key, nil *G2): Combine's identity;
//   - a point, kept as its 128-byte marshal (reduced, as upstream Marshal
//     writes it), optionally annotated with its registry index;
//   - a lazy registry aggregate: the set of registry indices whose keys it
//     sums. Combine over registry keys only ORs bits; VerifySignature then
//     runs the fold and the check on the GPU in one request (the batched
//     verifySignature of processing.go:342-368 without touching Handel).
type PublicKey struct {
	e *Engine
	// point form
	p []byte
	// registry binding: idx >= 0 for a registry key; bits != nil for an aggregate
	reg  *Registry
	idx  int
	bits []uint64
	// materialised marshal of an aggregate (computed once)
	aggOnce sync.Once
	agg     []byte
	aggErr  error
}

// bindRegistry annotates a key with its index in r (the latest load that
// holds it wins). Index-based use checks that the binding is usable: same
// engine, and r still the registry loaded on it (see indexed).
func (p *PublicKey) bindRegistry(r *Registry, i int) {
	p.reg = r
	p.idx = i
}

// indexed reports whether index-based requests for this key or aggregate are
// valid now: its registry is the one loaded on the key's own engine. The
// caller holds p.e.regMu for reading until its request has run.
func (p *PublicKey) indexed() bool { return p.reg != nil && p.reg.e == p.e && p.reg.current() }

func (p *PublicKey) isEmpty() bool { return p.p == nil && p.bits == nil }

func (p *PublicKey) lazy() bool { return p.bits != nil }

// registryBits returns the key as a set of registry indices, if it is one.
func (p *PublicKey) registryBits() ([]uint64, *Registry, bool) {
	if p.reg == nil {
		return nil, nil, false
	}
	if p.bits != nil {
		return p.bits, p.reg, true
	}
	if p.p != nil && p.idx >= 0 {
		w := make([]uint64, (p.reg.size+63)/64)
		w[p.idx>>6] |= 1 << uint(p.idx&63)
		return w, p.reg, true
	}
	return nil, nil, false
}

// point returns the 128-byte marshal, folding a lazy aggregate on the GPU.
func (p *PublicKey) point() ([]byte, error) {
	if !p.lazy() {
		return p.p, nil
	}
	p.aggOnce.Do(func() {
		p.e.regMu.RLock()
		defer p.e.regMu.RUnlock()
		if !p.indexed() {
			// the registry was replaced (or belongs to another engine): fold its points
			p.agg, p.aggErr = p.reg.foldPoints(p.e, p.bits)
			return
		}
		n := p.reg.size
		out, codes, err := p.e.AggregateKeys([]Request{{Offset: 0, LevelSize: n, BitLen: n, Words: p.bits}})
		if err == nil {
			err = p.e.CodeError(codes[0])
		}
		p.agg, p.aggErr = out, err
	})
	return p.agg, p.aggErr
}

// String implements handel.PublicKey: hex of the marshal (go flavor), hex of
// its SHA-256 (cf flavor, bn256/cf/bn256.go:75-80).
func (p *PublicKey) String() string {
	b, err := p.MarshalBinary()
	if err != nil {
		return "<nil>"
	}
	if p.e.flavor == FlavorCF {
		s := sha256.Sum256(b)
		return hex.EncodeToString(s[:])
	}
	return hex.EncodeToString(b)
}

// MarshalBinary implements the simul/lib PublicKey interface.
func (p *PublicKey) MarshalBinary() ([]byte, error) {
	if p.isEmpty() {
		return nil, errors.New("hip: nil public key")
	}
	b, err := p.point()
	if err != nil {
		return nil, err
	}
	out := make([]byte, len(b))
	copy(out, b)
	return out, nil
}

// UnmarshalBinary implements the simul/lib PublicKey interface with the
// flavor's rules and error texts (go: "unable to unmarshal",
// bn256/go/bn256.go:113-120; cf: the cloudflare error as is, :117-121). The
// point is decoded and re-encoded on the GPU (a sum with infinity).
func (p *PublicKey) UnmarshalBinary(buff []byte) error {
	if p.e.flavor == FlavorGo && len(buff) != 128 {
		return errors.New("unable to unmarshal")
	}
	if p.e.flavor == FlavorCF && len(buff) < 128 {
		return errors.New("bn256: not enough data")
	}
	out, codes, err := p.e.CombineG2(buff[:128], make([]byte, 128))
	if err != nil {
		return err
	}
	if err := p.e.CodeError(codes[0]); err != nil {
		return err
	}
	*p = PublicKey{e: p.e, p: out, idx: -1}
	return nil
}

// Combine implements handel.PublicKey (bn256/go/bn256.go:97-105): a nil
// receiver returns the argument; otherwise a fresh key, inputs untouched. A
// type mismatch panics like the reference's type assertion.
func (p *PublicKey) Combine(pp handel.PublicKey) handel.PublicKey {
	if p.isEmpty() {
		return pp
	}
	p2 := pp.(*PublicKey)
	if a, ra, ok := p.registryBits(); ok && ra.e == p.e {
		if b, rb, ok2 := p2.registryBits(); ok2 && ra == rb && p2.e == p.e {
			w := make([]uint64, len(a))
			disjoint := true
			for i := range a {
				if a[i]&b[i] != 0 {
					disjoint = false
					break
				}
				w[i] = a[i] | b[i]
			}
			// a key combined twice is 2*pk, not a set union: only disjoint
			// index sets stay lazy
			if disjoint {
				return &PublicKey{e: p.e, reg: ra, idx: -1, bits: w}
			}
		}
	}
	x, err := p.point()
	if err != nil {
		panic(err)
	}
	y, err := p2.point()
	if err != nil {
		panic(err)
	}
	out, codes, err := p.e.CombineG2(x, y)
	if err != nil {
		panic(err)
	}
	if err := p.e.CodeError(codes[0]); err != nil {
		panic(err)
	}
	return &PublicKey{e: p.e, p: out, idx: -1}
}

// VerifySignature implements handel.PublicKey (bn256/go/bn256.go:82-94):
// nil, "bn256: signature invalid", or the hash error ("EOF"). The check is
// e(H(m), pk) * e(-sig, G2Base) == 1 with one final exponentiation, which
// gives the reference's verdict for every pk in G2 (DESIGN.md §1). Calls are
// queued on the engine's batcher, so concurrent callers share a launch.
//
// Deviation: an empty key makes the reference dereference a nil point and
// panic; here it returns that runtime error's text as an error.
func (p *PublicKey) VerifySignature(msg []byte, sig handel.Signature) error {
	ms := sig.(*SigBLS)
	if p.isEmpty() {
		return p.e.CodeError(codeEmptyAgg)
	}
	s, err := ms.MarshalBinary()
	if err != nil {
		return err
	}
	if p.lazy() || (p.reg != nil && p.idx >= 0) {
		// index-based requests only while the key's registry is the one loaded
		// on its engine (held for reading until the request has run)
		p.e.regMu.RLock()
		if p.indexed() {
			defer p.e.regMu.RUnlock()
			if p.lazy() {
				n := p.reg.size
				return p.e.submit(msg, &Request{Offset: 0, LevelSize: n, BitLen: n, Words: p.bits, Sig: s}, nil)
			}
			// a registry key (the p2p aggregator's verifyPacket, simul/p2p/aggregator.go:244):
			// a one-key aggregate request, so the check uses the precomputed e(H, pk)
			return p.e.submit(msg, &Request{Offset: p.idx, LevelSize: 1, BitLen: 1, Words: []uint64{1}, Sig: s}, nil)
		}
		p.e.regMu.RUnlock()
	}
	pt, err := p.point() // the point path: a key outside the loaded registry, or a stale aggregate
	if err != nil {
		return err
	}
	return p.e.submit(msg, nil, &single{pk: pt, sig: s})
}

// SecretKey is the secret scalar (bn256/go/bn256.go:122-166).
type SecretKey struct {
	e *Engine
	s *big.Int
}

func scalar32(k *big.Int) []byte {
	b := k.Bytes()
	out := make([]byte, 32)
	copy(out[32-len(b):], b)
	return out
}

// NewKeyPair is bn256/go/bn256.go:129-142 on the default go-flavor engine:
// k = crypto/rand.Int(reader, Order) until k > 0 (x/crypto RandomG2), pk = k*G2.
func NewKeyPair(reader io.Reader) (*SecretKey, *PublicKey, error) {
	e, err := Default(FlavorGo)
	if err != nil {
		return nil, nil, err
	}
	return newKeyPair(e, reader)
}

func newKeyPair(e *Engine, reader io.Reader) (*SecretKey, *PublicKey, error) {
	if reader == nil {
		reader = rand.Reader
	}
	var k *big.Int
	for {
		var err error
		k, err = rand.Int(reader, Order)
		if err != nil {
			return nil, nil, err
		}
		if k.Sign() > 0 {
			break
		}
	}
	pk, err := e.Keygen(scalar32(k))
	if err != nil {
		return nil, nil, err
	}
	return &SecretKey{e: e, s: k}, &PublicKey{e: e, p: pk, idx: -1}, nil
}

// Sign implements handel.SecretKey: sig = s*H(msg) (bn256/go/bn256.go:146-154).
func (s *SecretKey) Sign(msg []byte, reader io.Reader) (handel.Signature, error) {
	out, err := s.e.Sign(msg, scalar32(s.s))
	if err != nil {
		return nil, err
	}
	return &SigBLS{e: s.e, b: out}, nil
}

// MarshalBinary is big.Int.Bytes() (bn256/go/bn256.go:157-159).
func (s *SecretKey) MarshalBinary() ([]byte, error) { return s.s.Bytes(), nil }

// UnmarshalBinary is big.Int.SetBytes (bn256/go/bn256.go:162-166).
func (s *SecretKey) UnmarshalBinary(buff []byte) error {
	s.s = new(big.Int).SetBytes(buff)
	return nil
}

// SigBLS is a BLS signature, a G1 point kept as its 64-byte marshal
// (bn256/go/bn256.go:168-204).
type SigBLS struct {
	e *Engine
	b []byte
}

// MarshalBinary implements handel.Signature.
func (m *SigBLS) MarshalBinary() ([]byte, error) {
	if m.b == nil {
		return nil, errors.New("bn256: multisig can't marshal if nil")
	}
	out := make([]byte, 64)
	copy(out, m.b)
	return out, nil
}

// UnmarshalBinary implements handel.Signature with the flavor's rules and
// texts: go "bn256: multisig can't unmarshal" (bn256/go/bn256.go:182-189);
// cf "bn256: multisig can't unmarshal: <cloudflare error>"
// (bn256/cf/bn256.go:183-190).
func (m *SigBLS) UnmarshalBinary(b []byte) error {
	if m.e.flavor == FlavorGo && len(b) != 64 {
		return errors.New("bn256: multisig can't unmarshal")
	}
	if m.e.flavor == FlavorCF && len(b) < 64 {
		return errors.New("bn256: multisig can't unmarshal: bn256: not enough data")
	}
	out, codes, err := m.e.CombineG1(b[:64], make([]byte, 64))
	if err != nil {
		return err
	}
	if err := m.e.CodeError(codes[0]); err != nil {
		return err
	}
	m.b = out
	return nil
}

// Combine implements handel.Signature (bn256/go/bn256.go:192-200).
func (m *SigBLS) Combine(ms handel.Signature) handel.Signature {
	if m.b == nil {
		return ms
	}
	m2 := ms.(*SigBLS)
	out, codes, err := m.e.CombineG1(m.b, m2.b)
	if err != nil {
		panic(err)
	}
	if err := m.e.CodeError(codes[0]); err != nil {
		panic(err)
	}
	return &SigBLS{e: m.e, b: out}
}

func (m *SigBLS) String() string { return hex.EncodeToString(m.b) }
