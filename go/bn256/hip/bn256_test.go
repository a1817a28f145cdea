package hip

// The reference's property tests for its bn256 plugins
// (bn256/go/bn256_test.go:39-103), on the MI355X engine, plus the batched
// paths against the one-at-a-time ones. Needs a GPU and libhandel_gpu.so;
// not compiled here (no Go toolchain) — tests/test_gpu_boundary.py and
// tests/native/abi_threads.c cover the same C calls from Python and C.

import (
	"crypto/rand"
	"sync"
	"testing"
	"time"

	h "github.com/ConsenSys/handel"
	"github.com/stretchr/testify/require"
)

var funky = []byte("Get Funky Tonight")

// TestHandel is the reference's in-protocol test (bn256/go/bn256_test.go:13-37):
// 37 Handel instances with real BLS reach the full multisignature. Here the
// keys are hip keys, loaded as the engine's registry before the run, so every
// Combine Handel does over registry keys stays a bitset and every
// verifySignature (processing.go:342-368) becomes one aggregate request of the
// engine's batcher; the GT tables are prepared for the message.
func TestHandel(t *testing.T) {
	n := 37
	config := h.DefaultConfig(n)
	msg := []byte("Peaches and Cream")
	e, err := NewEngine(0, FlavorGo)
	require.NoError(t, err)
	defer e.Close()
	cons := NewConstructorOn(e)
	secretKeys := make([]h.SecretKey, n)
	pubKeys := make([]h.PublicKey, n)
	ids := make([]h.Identity, n)
	for i := 0; i < n; i++ {
		sec, pub := cons.KeyPair(rand.Reader)
		secretKeys[i] = sec
		pubKeys[i] = pub
		// the identities NewTest builds (test.go:35-47): same ids, same key objects
		ids[i] = h.NewStaticIdentity(int32(i), "", pub)
	}
	_, err = e.LoadRegistry(h.NewArrayRegistry(ids))
	require.NoError(t, err)
	require.NoError(t, e.PrepareAggregate(msg))
	test := h.NewTest(secretKeys, pubKeys, cons, msg, config)
	test.Start()
	defer test.Stop()

	select {
	case <-test.WaitCompleteSuccess():
	case <-time.After(100 * time.Second):
		t.FailNow()
	}
}

// A registry replaced on its engine: keys and lazy aggregates bound to the old
// one must not be checked by index against the new one (they take the point
// path), and the old Registry's batched entry points refuse to run.
func TestRegistryReplaced(t *testing.T) {
	e, err := NewEngine(0, FlavorGo)
	require.NoError(t, err)
	defer e.Close()
	regA, sksA, rA := testRegistry(t, e, 16)
	_, _, rB := testRegistry(t, e, 16) // replaces A on the engine
	require.False(t, rA.current())
	require.True(t, rB.current())
	id3, _ := regA.Identity(3)
	id5, _ := regA.Identity(5)
	s3, _ := sksA[3].Sign(funky, nil)
	s5, _ := sksA[5].Sign(funky, nil)
	require.NoError(t, id3.PublicKey().VerifySignature(funky, s3))
	agg := id3.PublicKey().Combine(id5.PublicKey())
	require.True(t, agg.(*PublicKey).lazy())
	require.NoError(t, agg.VerifySignature(funky, s3.Combine(s5)))
	require.EqualError(t, id3.PublicKey().VerifySignature(funky, s5), "bn256: signature invalid")
	bs := h.NewWilffBitset(16)
	bs.Set(3, true)
	errs := rA.VerifyMultiSignatures(funky, []*h.MultiSignature{{BitSet: bs, Signature: s3}})
	require.EqualError(t, errs[0], "hip: registry is no longer loaded on its engine")
}

// A key bound to a registry of another engine is checked by its point.
func TestKeyOfOtherEngine(t *testing.T) {
	a, err := NewEngine(0, FlavorGo)
	require.NoError(t, err)
	defer a.Close()
	b, err := NewEngine(0, FlavorGo)
	require.NoError(t, err)
	defer b.Close()
	regA, sksA, _ := testRegistry(t, a, 8)
	id2, _ := regA.Identity(2)
	// the same key objects loaded on engine b: bound to b's registry now
	ids := make([]h.Identity, 8)
	for i := range ids {
		ids[i], _ = regA.Identity(i)
	}
	_, err = b.LoadRegistry(h.NewArrayRegistry(ids))
	require.NoError(t, err)
	s2, _ := sksA[2].Sign(funky, nil)
	require.NoError(t, id2.PublicKey().VerifySignature(funky, s2)) // key of engine a, registry of b: point path
}

// Range checks every identity of a level slice.
func TestRegistryRangeContiguous(t *testing.T) {
	e, err := NewEngine(0, FlavorGo)
	require.NoError(t, err)
	defer e.Close()
	reg, _, r := testRegistry(t, e, 16)
	slice := func(ix ...int) []h.Identity {
		out := make([]h.Identity, len(ix))
		for j, i := range ix {
			out[j], _ = reg.Identity(i)
		}
		return out
	}
	off, err := r.Range(slice(4, 5, 6, 7))
	require.NoError(t, err)
	require.Equal(t, 4, off)
	_, err = r.Range(slice(4, 9, 6, 7)) // right endpoints, wrong middle
	require.Error(t, err)
	_, err = r.Range(slice(14, 15, 16))
	require.Error(t, err)
}

func TestSign(t *testing.T) {
	sk, pk, err := NewKeyPair(rand.Reader)
	require.NoError(t, err)
	sig, err := sk.Sign(funky, nil)
	require.NoError(t, err)
	buff, _ := sig.MarshalBinary()
	require.Len(t, buff, 64)
	buff, _ = pk.MarshalBinary()
	require.Len(t, buff, 128)
	require.NoError(t, pk.VerifySignature(funky, sig))
	// a message whose digest is >= n cannot be hashed (hashedMessage: EOF)
	_, err = sk.Sign([]byte("hello world"), nil)
	require.EqualError(t, err, "EOF")
}

func TestCombine(t *testing.T) {
	sk1, pk1, err := NewKeyPair(rand.Reader)
	require.NoError(t, err)
	sk2, pk2, err := NewKeyPair(rand.Reader)
	require.NoError(t, err)
	require.NotEqual(t, pk1.String(), pk2.String())
	sig1, err := sk1.Sign(funky, nil)
	require.NoError(t, err)
	require.NoError(t, pk1.VerifySignature(funky, sig1))
	sig2, err := sk2.Sign(funky, nil)
	require.NoError(t, err)
	require.NoError(t, pk2.VerifySignature(funky, sig2))
	sig3 := sig1.Combine(sig2)
	pk3 := pk1.Combine(pk2)
	require.NoError(t, pk3.VerifySignature(funky, sig3))
	require.EqualError(t, pk1.VerifySignature(funky, sig2), "bn256: signature invalid")
}

func TestMarshalling(t *testing.T) {
	sk, pk, err := NewKeyPair(nil)
	require.NoError(t, err)
	buffSK, err := sk.MarshalBinary()
	require.NoError(t, err)
	buffPK, err := pk.MarshalBinary()
	require.NoError(t, err)
	cons := NewConstructor()
	sk2 := cons.SecretKey()
	require.NoError(t, sk2.(*SecretKey).UnmarshalBinary(buffSK))
	pk2 := cons.PublicKey()
	require.NoError(t, pk2.(*PublicKey).UnmarshalBinary(buffPK))
	require.Equal(t, pk.String(), pk2.String())
	require.EqualError(t, cons.Signature().UnmarshalBinary(make([]byte, 63)), "bn256: multisig can't unmarshal")
	require.EqualError(t, cons.PublicKey().(*PublicKey).UnmarshalBinary(make([]byte, 127)), "unable to unmarshal")
	cf := NewConstructorCF()
	require.EqualError(t, cf.Signature().UnmarshalBinary(make([]byte, 63)),
		"bn256: multisig can't unmarshal: bn256: not enough data")
}

// registry of n keys on engine e, with their secret keys
func testRegistry(t *testing.T, e *Engine, n int) (h.Registry, []h.SecretKey, *Registry) {
	cons := NewConstructorOn(e)
	ids := make([]h.Identity, n)
	sks := make([]h.SecretKey, n)
	for i := range ids {
		sk, pk := cons.KeyPair(rand.Reader)
		ids[i] = h.NewStaticIdentity(int32(i), "", pk)
		sks[i] = sk
	}
	reg := h.NewArrayRegistry(ids)
	r, err := e.LoadRegistry(reg)
	require.NoError(t, err)
	return reg, sks, r
}

// The lazy registry aggregate (Combine over registry keys keeps a bitset)
// verifies exactly like the explicit point fold.
func TestLazyAggregate(t *testing.T) {
	e, err := NewEngine(0, FlavorGo)
	require.NoError(t, err)
	defer e.Close()
	reg, sks, _ := testRegistry(t, e, 100)
	cons := NewConstructorOn(e)
	agg := cons.PublicKey()
	sig := cons.Signature()
	explicit := cons.PublicKey()
	for i := 0; i < 100; i += 3 {
		id, _ := reg.Identity(i)
		agg = agg.Combine(id.PublicKey())
		b, _ := id.PublicKey().(*PublicKey).MarshalBinary()
		pk := cons.PublicKey().(*PublicKey)
		require.NoError(t, pk.UnmarshalBinary(b)) // not a registry key: explicit path
		explicit = explicit.Combine(pk)
		s, err := sks[i].Sign(funky, nil)
		require.NoError(t, err)
		sig = sig.Combine(s)
	}
	require.True(t, agg.(*PublicKey).lazy())
	require.NoError(t, agg.VerifySignature(funky, sig))
	a, _ := agg.(*PublicKey).MarshalBinary()
	b, _ := explicit.(*PublicKey).MarshalBinary()
	require.Equal(t, b, a)
	// a key combined twice is 2*pk: leaves the lazy form, still correct
	id0, _ := reg.Identity(0)
	twice := agg.Combine(id0.PublicKey())
	require.False(t, twice.(*PublicKey).lazy())
}

// Concurrent VerifySignature callers (k instances per process) are merged by
// the batcher and each gets its own verdict.
func TestBatcherConcurrent(t *testing.T) {
	_, pk, _ := NewKeyPair(nil)
	sk2, _, _ := NewKeyPair(nil)
	var wg sync.WaitGroup
	for g := 0; g < 32; g++ {
		wg.Add(1)
		go func(g int) {
			defer wg.Done()
			sk, pkg, err := NewKeyPair(nil)
			require.NoError(t, err)
			sig, _ := sk.Sign(funky, nil)
			bad, _ := sk2.Sign(funky, nil)
			for i := 0; i < 8; i++ {
				require.NoError(t, pkg.VerifySignature(funky, sig))
				require.EqualError(t, pk.VerifySignature(funky, bad), "bn256: signature invalid")
			}
		}(g)
	}
	wg.Wait()
}

// VerifyMultiSignatures: size mismatch text and a valid full-registry check.
func TestVerifyMultiSignatures(t *testing.T) {
	e, err := NewEngine(0, FlavorGo)
	require.NoError(t, err)
	defer e.Close()
	_, sks, r := testRegistry(t, e, 40)
	bs := h.NewWilffBitset(40)
	cons := NewConstructorOn(e)
	sig := cons.Signature()
	for i := 0; i < 40; i += 2 {
		bs.Set(i, true)
		s, _ := sks[i].Sign(funky, nil)
		sig = sig.Combine(s)
	}
	short := h.NewWilffBitset(39)
	errs := r.VerifyMultiSignatures(funky, []*h.MultiSignature{
		{BitSet: bs, Signature: sig},
		{BitSet: short, Signature: sig},
	})
	require.NoError(t, errs[0])
	require.EqualError(t, errs[1], "verify multisignature: inconsistent sizes")
}
