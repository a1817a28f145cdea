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
	if _, err := e.loadRegistry(buf); err != nil {
		return nil, err
	}
	r := &Registry{e: e, size: n, index: index}
	for i, pk := range keys {
		pk.bindRegistry(r, i)
	}
	e.regMu.Lock()
	e.reg = r
	e.regMu.Unlock()
	return r, nil
}

// Size is the number of registry keys.
func (r *Registry) Size() int { return r.size }

// Range maps a level's identities (Partitioner.IdentitiesAt, a contiguous
// registry slice by partitioner.go:133-178) to its registry offset.
func (r *Registry) Range(ids []handel.Identity) (offset int, err error) {
	if len(ids) == 0 {
		return 0, nil
	}
	lo, ok := r.index[ids[0].ID()]
	hi, ok2 := r.index[ids[len(ids)-1].ID()]
	if !ok || !ok2 || hi-lo != len(ids)-1 {
		return 0, errors.New("hip: level identities are not a contiguous registry range")
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
