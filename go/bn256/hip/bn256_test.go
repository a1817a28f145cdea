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

	h "github.com/ConsenSys/handel"
	"github.com/stretchr/testify/require"
)

var funky = []byte("Get Funky Tonight")

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
