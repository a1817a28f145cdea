package hip

import "sync"

// single is one independent check: a 128-byte key marshal and a 64-byte
// signature marshal.
type single struct {
	pk, sig []byte
}

type job struct {
	msg  []byte
	agg  *Request
	one  *single
	done chan error
}

// batcher merges concurrent PublicKey.VerifySignature calls into launches
// (SURVEY.md §8(b) option 1: no Handel change). One goroutine takes the
// first queued job, drains whatever else is queued (up to maxBatch), groups
// the jobs by message and kind, and submits each group as one C call. There
// is no timer: while one launch runs the next batch accumulates, so the batch
// width follows the number of concurrent callers (k Handel instances per
// process, simul/node/main.go:63-131) without adding latency to a lone caller.
type batcher struct {
	e  *Engine
	ch chan *job
	wg sync.WaitGroup
}

const maxBatch = 4096

func (e *Engine) batch() *batcher {
	e.bOnce.Do(func() {
		e.b = &batcher{e: e, ch: make(chan *job, maxBatch)}
		e.b.wg.Add(1)
		go e.b.run()
	})
	return e.b
}

// submit queues one check and waits for its verdict (the error
// PublicKey.VerifySignature returns).
func (e *Engine) submit(msg []byte, agg *Request, one *single) error {
	j := &job{msg: msg, agg: agg, one: one, done: make(chan error, 1)}
	e.batch().ch <- j
	return <-j.done
}

func (b *batcher) run() {
	defer b.wg.Done()
	for {
		j, ok := <-b.ch
		if !ok {
			return
		}
		jobs := []*job{j}
	drain:
		for len(jobs) < maxBatch {
			select {
			case j2, ok := <-b.ch:
				if !ok {
					break drain
				}
				jobs = append(jobs, j2)
			default:
				break drain
			}
		}
		b.flush(jobs)
	}
}

type groupKey struct {
	msg string
	agg bool
}

func (b *batcher) flush(jobs []*job) {
	groups := map[groupKey][]*job{}
	var order []groupKey
	for _, j := range jobs {
		k := groupKey{string(j.msg), j.agg != nil}
		if _, ok := groups[k]; !ok {
			order = append(order, k)
		}
		groups[k] = append(groups[k], j)
	}
	for _, k := range order {
		g := groups[k]
		msg := []byte(k.msg)
		var codes []int32
		var err error
		if k.agg {
			reqs := make([]Request, len(g))
			for i, j := range g {
				reqs[i] = *j.agg
			}
			codes, _, err = b.e.VerifyAggregate(msg, reqs, false)
		} else {
			pks := make([]byte, 0, 128*len(g))
			sigs := make([]byte, 0, 64*len(g))
			for _, j := range g {
				pks = append(pks, j.one.pk...)
				sigs = append(sigs, j.one.sig...)
			}
			codes, err = b.e.VerifyBatch(msg, pks, sigs)
		}
		for i, j := range g {
			if err != nil {
				j.done <- err // the whole submission failed: no verdict, not "valid"
			} else {
				j.done <- b.e.CodeError(codes[i])
			}
		}
	}
}

func (b *batcher) close() {
	close(b.ch)
	b.wg.Wait()
}
