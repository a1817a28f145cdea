//go:build handel_batch

package hip

// TestHandel through the batched evaluator (SURVEY.md §8(b) option 2): with
// go/handel/config_hook.patch and go/handel/batched_processing.go applied to
// the Handel tree, Config.BatchVerifier routes every instance's checks
// through Registry.VerifyBatch, K = VerifyBatchSize per call. Build with
// -tags handel_batch (the hook is not part of upstream Handel).

import (
	"crypto/rand"
	"testing"
	"time"

	h "github.com/ConsenSys/handel"
	"github.com/stretchr/testify/require"
)

func TestHandelBatched(t *testing.T) {
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
		secretKeys[i], pubKeys[i] = sec, pub
		ids[i] = h.NewStaticIdentity(int32(i), "", pub)
	}
	r, err := e.LoadRegistry(h.NewArrayRegistry(ids))
	require.NoError(t, err)
	require.NoError(t, e.PrepareAggregate(msg))
	config.BatchVerifier = r
	config.VerifyBatchSize = 8
	test := h.NewTest(secretKeys, pubKeys, cons, msg, config)
	test.Start()
	defer test.Stop()
	select {
	case <-test.WaitCompleteSuccess():
	case <-time.After(100 * time.Second):
		t.FailNow()
	}
}
