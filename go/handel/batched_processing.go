package handel

// Batched signature processing: the drop-in replacement of
// evaluatorProcessing (processing.go:91-287) for verifiers that check many
// signatures per call (the MI355X engine, package bn256/hip). This file is
// added to the Handel package; config_hook.patch selects it from NewHandel
// when Config.BatchVerifier is set. Go is not installed where it was
// written, so it has not been compiled.
//
// Semantics: readTodos keeps the reference's scan (every todo evaluated once
// per pass, zero marks dropped, the death pill stops the loop) but keeps the
// K best marks instead of one; with K = 1 the pick and the queue order are
// exactly the reference's. Each pass verifies its slots in ONE BatchVerifier
// call and publishes the valid ones in slot order. Verdicts are a pure
// function of (msg, level range, bitset, signature), so batching cannot
// change them; the error of a request is the one verifySignature returns.

import (
	"sync"
	"time"
)

// BatchRequest is one verifySignature call (processing.go:342-368): the
// identities of the signature's level (Partitioner.IdentitiesAt, a
// contiguous registry range) and the multisignature.
type BatchRequest struct {
	Level      int
	Identities []Identity
	MultiSig   *MultiSignature
}

// BatchVerifier verifies many requests at once. It returns one error per
// request: nil, or exactly the error verifySignature would return
// ("handel: inconsistent bitset with given level", "handel: <VerifySignature
// error>"). A failure of the whole call is reported as that error for every
// request, never as nil.
type BatchVerifier interface {
	VerifyBatch(msg []byte, reqs []BatchRequest) []error
}

// DefaultVerifyBatchSize is K when Config.VerifyBatchSize is 0.
const DefaultVerifyBatchSize = 16

type slot struct {
	mark int
	sig  *incomingSig
}

type batchedProcessing struct {
	cond *sync.Cond

	part     Partitioner
	msg      []byte
	out      chan incomingSig
	todos    []*incomingSig
	eval     SigEvaluator
	log      Logger
	filter   Filter
	verifier BatchVerifier
	k        int

	// the reference's statistics (processing.go:107-118), per signature
	sigCheckedCt    int
	sigQueueSize    int
	sigSuppressed   int
	sigCheckingTime int
	batches         int
}

func newBatchedProcessing(part Partitioner, msg []byte, e SigEvaluator, log Logger, v BatchVerifier, k int) signatureProcessing {
	if k <= 0 {
		k = DefaultVerifyBatchSize
	}
	m := sync.Mutex{}
	return &batchedProcessing{
		cond:     sync.NewCond(&m),
		part:     part,
		msg:      msg,
		out:      make(chan incomingSig, 1000),
		todos:    make([]*incomingSig, 0),
		eval:     e,
		log:      log,
		filter:   newIndividualSigFilter(),
		verifier: v,
		k:        k,
	}
}

func (f *batchedProcessing) Start() { go f.processLoop() }

func (f *batchedProcessing) Stop() { f.Add(&deathPillPair) }

func (f *batchedProcessing) Verified() chan incomingSig { return f.out }

func (f *batchedProcessing) Add(sp *incomingSig) {
	f.cond.L.Lock()
	defer f.cond.L.Unlock()
	if f.filter.Accept(sp) {
		f.todos = append(f.todos, sp)
		f.cond.Signal()
	}
}

// readTodos is processing.go:171-220 with `best` widened to K slots sorted by
// descending mark (ties keep arrival order). A todo that does not make the
// slots, or is pushed out of them, goes back to the queue in scan order.
func (f *batchedProcessing) readTodos() (bool, []*incomingSig) {
	f.cond.L.Lock()
	defer f.cond.L.Unlock()
	for len(f.todos) == 0 {
		f.cond.Wait()
	}
	previousLen := len(f.todos)
	var newTodos []*incomingSig
	slots := make([]slot, 0, f.k)
	for _, pair := range f.todos {
		if *pair == deathPillPair {
			return true, nil
		}
		if pair.ms == nil {
			continue
		}
		mark := f.eval.Evaluate(pair)
		if mark <= 0 {
			continue
		}
		if len(slots) == f.k && mark <= slots[len(slots)-1].mark {
			newTodos = append(newTodos, pair)
			continue
		}
		if len(slots) == f.k {
			newTodos = append(newTodos, slots[len(slots)-1].sig)
			slots = slots[:len(slots)-1]
		}
		j := len(slots)
		for j > 0 && slots[j-1].mark < mark {
			j--
		}
		slots = append(slots, slot{})
		copy(slots[j+1:], slots[j:])
		slots[j] = slot{mark, pair}
	}
	f.todos = newTodos
	newLen := len(f.todos)
	f.sigSuppressed += previousLen - newLen - len(slots)
	f.sigCheckedCt += len(slots)
	f.sigQueueSize += newLen * len(slots)
	batch := make([]*incomingSig, len(slots))
	for i, s := range slots {
		batch[i] = s.sig
	}
	return false, batch
}

func (f *batchedProcessing) processLoop() {
	for {
		done, batch := f.readTodos()
		if done {
			close(f.out)
			return
		}
		if len(batch) > 0 {
			f.verifyAndPublish(batch)
		}
	}
}

// verifyAndPublish is processing.go:270-287 for a whole batch: one verifier
// call, valid signatures sent on `out` in slot order, the others logged as
// Warn("verify", err).
func (f *batchedProcessing) verifyAndPublish(batch []*incomingSig) {
	start := time.Now()
	errs := make([]error, len(batch))
	reqs := make([]BatchRequest, 0, len(batch))
	where := make([]int, 0, len(batch))
	for i, sp := range batch {
		ids, err := f.part.IdentitiesAt(int(sp.level))
		if err != nil {
			errs[i] = err // verifySignature returns it as is (processing.go:345-348)
			continue
		}
		reqs = append(reqs, BatchRequest{Level: int(sp.level), Identities: ids, MultiSig: sp.ms})
		where = append(where, i)
	}
	if len(reqs) > 0 {
		res := f.verifier.VerifyBatch(f.msg, reqs)
		for j, i := range where {
			errs[i] = res[j]
		}
	}
	// the reference accumulates whole milliseconds per check; a batch's time
	// is shared by its checks
	f.sigCheckingTime += int(time.Since(start).Nanoseconds() / 1000000)
	f.batches++
	for i, sp := range batch {
		if errs[i] != nil {
			f.log.Warn("verify", errs[i])
		} else {
			f.out <- *sp
		}
	}
}

// Values implements Reporter with the reference's keys (processing.go:241-256)
// plus the batch count.
func (f *batchedProcessing) Values() map[string]float64 {
	sigQueueSize, sigCheckingTime, batchWidth := 0.0, 0.0, 0.0
	if f.sigCheckedCt > 0 {
		sigQueueSize = float64(f.sigQueueSize) / float64(f.sigCheckedCt)
		sigCheckingTime = float64(f.sigCheckingTime) / float64(f.sigCheckedCt)
	}
	if f.batches > 0 {
		batchWidth = float64(f.sigCheckedCt) / float64(f.batches)
	}
	return map[string]float64{
		"sigCheckedCt":    float64(f.sigCheckedCt),
		"sigQueueSize":    sigQueueSize,
		"sigSuppressed":   float64(f.sigSuppressed),
		"sigCheckingTime": sigCheckingTime,
		"sigBatches":      float64(f.batches),
		"sigBatchWidth":   batchWidth,
	}
}
