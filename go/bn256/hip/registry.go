package hip

import (
	"errors"
	"fmt"

	"github.com/ConsenSys/handel"
)

// Registry is the device-resident copy of a Handel registry
// (identity.go:22-31): every key decoded once on the GPU
// (PublicKey.UnmarshalBinary for N keys, simul/lib/nodes.go:44-64), plus the
// window subset sums and power-of-two block sums the aggregate fold reads.
// Registry keys (*PublicKey) learn their index, so Combine over them can stay
// a bitset until VerifySignature (see PublicKey).
type Registry struct {
	e     *Engine
	size  int
	index map[int32]int // identity ID -> registry index
	keys  [][]byte      // the key marshals, for folds once this registry is no longer loaded
}

// LoadRegistry uploads reg to the engine. Every identity's PublicKey must be
// a *PublicKey of this package; the keys are annotated in place with their
// registry index (a read-only annotation: the point itself never changes).
func (e *Engine) LoadRegistry(reg handel.Registry) (*Registry, error) {
	n := reg.Size()
	buf := make([]byte, 0, 128*n)
	keys := make([]*PublicKey, n)
	index := make(map[int32]int, n)
	for i := 0; i < n; i++ {
		id, ok := reg.Identity(i)
		if !ok {
			return nil, fmt.Errorf("registry returned empty identity at %d", i)
		}
		pk, ok := id.PublicKey().(*PublicKey)
		if !ok {
			return nil, errors.New("hip: registry key is not a hip.PublicKey")
		}
		b, err := pk.MarshalBinary()
		if err != nil {
			return nil, err
		}
		buf = append(buf, b...)
		keys[i] = pk
		index[id.ID()] = i
	}
	// the load replaces the context's registry: no index-based check may run
	// against it meanwhile (they hold regMu for reading, see current)
	e.regMu.Lock()
	defer e.regMu.Unlock()
	e.reg = nil
	if _, err := e.loadRegistry(buf); err != nil {
		return nil, err
	}
	marshals := make([][]byte, n)
	for i := range marshals {
		marshals[i] = buf[128*i : 128*i+128]
	}
	r := &Registry{e: e, size: n, index: index, keys: marshals}
	for i, pk := range keys {
		pk.bindRegistry(r, i)
	}
	e.reg = r
	return r, nil
}

// current reports whether r is the registry its engine's context holds now,
// so index-based requests against the context mean r's keys. The caller must
// hold r.e.regMu (for reading) until its request has run.
func (r *Registry) current() bool { return r != nil && r.e.reg == r }

// foldPoints sums the keys whose bits are set with point additions (batched
// PublicKey.Combine, pairwise tree), for a lazy aggregate whose registry is no
// longer the loaded one.
func (r *Registry) foldPoints(e *Engine, bits []uint64) ([]byte, error) {
	var pts [][]byte
	for i := 0; i < r.size; i++ {
		if bits[i>>6]>>uint(i&63)&1 == 1 {
			pts = append(pts, r.keys[i])
		}
	}
	if len(pts) == 0 {
		return nil, e.CodeError(codeEmptyAgg)
	}
	for len(pts) > 1 {
		half := len(pts) / 2
		a := make([]byte, 0, 128*half)
		b := make([]byte, 0, 128*half)
		for i := 0; i < half; i++ {
			a = append(a, pts[2*i]...)
			b = append(b, pts[2*i+1]...)
		}
		out, codes, err := e.CombineG2(a, b)
		if err != nil {
			return nil, err
		}
		next := make([][]byte, 0, half+1)
		for i := 0; i < half; i++ {
			if err := e.CodeError(codes[i]); err != nil {
				return nil, err
			}
			next = append(next, out[128*i:128*i+128])
		}
		if len(pts)%2 == 1 {
			next = append(next, pts[len(pts)-1])
		}
		pts = next
	}
	return pts[0], nil
}

// Size is the number of registry keys.
func (r *Registry) Size() int { return r.size }

// Range maps a level's identities (Partitioner.IdentitiesAt, a contiguous
// registry slice by partitioner.go:133-178) to its registry offset. Every
// identity is checked: identity j must sit at registry index offset + j.
func (r *Registry) Range(ids []handel.Identity) (offset int, err error) {
	if len(ids) == 0 {
		return 0, nil
	}
	lo, ok := r.index[ids[0].ID()]
	if !ok || lo+len(ids) > r.size {
		return 0, errors.New("hip: level identities are not a contiguous registry range")
	}
	for j, id := range ids {
		if k, ok := r.index[id.ID()]; !ok || k != lo+j {
			return 0, errors.New("hip: level identities are not a contiguous registry range")
		}
	}
	return lo, nil
}

// bitsetWords converts a handel.BitSet into willf words (bit i = word[i>>6]
// bit i&63) by walking its set bits.
func bitsetWords(bs handel.BitSet) []uint64 {
	n := bs.BitLength()
	w := make([]uint64, (n+63)/64)
	for b, ok := bs.NextSet(0); ok && b < n; b, ok = bs.NextSet(b + 1) {
		w[b>>6] |= 1 << uint(b&63)
	}
	return w
}

// VerifyBatch implements handel.BatchVerifier (go/handel/batched_processing.go,
// added to Handel by go/handel/config_hook.patch): the batched
// verifySignature (processing.go:342-368) of every request in one
// hg_verify_aggregate launch — Combine fold over the level's set bits from
// the device-resident registry, then the pairing check. Errors are the
// reference's texts ("handel: inconsistent bitset with given level",
// "handel: bn256: signature invalid", "handel: EOF"). If the submission as a
// whole fails, every request gets that error: nothing is reported valid.
func (r *Registry) VerifyBatch(msg []byte, reqs []handel.BatchRequest) []error {
	out := make([]error, len(reqs))
	r.e.regMu.RLock()
	defer r.e.regMu.RUnlock()
	if !r.current() {
		// the engine has loaded another registry since: index-based requests
		// would check against its keys
		for i := range out {
			out[i] = errors.New("hip: registry is no longer loaded on its engine")
		}
		return out
	}
	creqs := make([]Request, 0, len(reqs))
	where := make([]int, 0, len(reqs))
	for i, q := range reqs {
		off, err := r.Range(q.Identities)
		if err != nil {
			out[i] = err
			continue
		}
		sig, err := q.MultiSig.Signature.(*SigBLS).MarshalBinary()
		if err != nil {
			out[i] = err
			continue
		}
		creqs = append(creqs, Request{
			Offset:    off,
			LevelSize: len(q.Identities),
			BitLen:    q.MultiSig.BitSet.BitLength(),
			Words:     bitsetWords(q.MultiSig.BitSet),
			Sig:       sig,
		})
		where = append(where, i)
	}
	if len(creqs) == 0 {
		return out
	}
	codes, _, err := r.e.VerifyAggregate(msg, creqs, false)
	for j, i := range where {
		if err != nil {
			out[i] = err
		} else {
			out[i] = r.e.ProcessingError(codes[j])
		}
	}
	return out
}

// VerifyMultiSignatures is crypto.go:120-137 VerifyMultiSignature for many
// multisignatures over this registry in one launch (the final-signature
// check of simul/node/main.go:127 and the p2p baselines). Each error is the
// reference's: "verify multisignature: inconsistent sizes" or the
// VerifySignature error.
func (r *Registry) VerifyMultiSignatures(msg []byte, ms []*handel.MultiSignature) []error {
	out := make([]error, len(ms))
	r.e.regMu.RLock()
	defer r.e.regMu.RUnlock()
	if !r.current() {
		for i := range out {
			out[i] = errors.New("hip: registry is no longer loaded on its engine")
		}
		return out
	}
	lens := make([]int, 0, len(ms))
	words := make([][]uint64, 0, len(ms))
	sigs := make([]byte, 0, 64*len(ms))
	where := make([]int, 0, len(ms))
	for i, m := range ms {
		s, err := m.Signature.(*SigBLS).MarshalBinary()
		if err != nil {
			out[i] = err
			continue
		}
		lens = append(lens, m.BitSet.BitLength())
		words = append(words, bitsetWords(m.BitSet))
		sigs = append(sigs, s...)
		where = append(where, i)
	}
	if len(where) == 0 {
		return out
	}
	codes, err := r.e.VerifyMultiSignatures(msg, lens, words, sigs)
	for j, i := range where {
		if err != nil {
			out[i] = err
		} else {
			out[i] = r.e.CodeError(codes[j])
		}
	}
	return out
}
