"""Batched signature processing: the drop-in for processing.go's
`signatureProcessing`.

The reference's `evaluatorProcessing` (processing.go:91-287) scores every
queued incoming signature with a `SigEvaluator`, keeps the rest, and verifies
ONE per loop iteration (`readTodos` picks the best, `verifyAndPublish` checks
it). `BatchedEvaluatorProcessing` keeps that interface — `start`, `stop`,
`add`, `verified` — and the same scoring, filtering and death-pill rules, but
`read_todos` returns the top-`batch` signatures (the reference's single-best
loop generalised to K slots; K = 1 reproduces the reference's pick and queue
order exactly) and the batch goes to the GPU in one launch through a
`verify` callable (normally `processing.BatchVerifier.verify_levels`, or a
`SharedBatcher` when several Handel instances share one GPU context, the
process model of simul/node/main.go:63-131).

`Store` mirrors the replace store's scoring and merging (store.go:39-260):
`evaluate` is `unsafeEvaluate` (store.go:111-183), the `EvaluatorStore`
strategy Handel runs with; `store` is `Store` + `unsafeCheckMerge`
(store.go:82-226), whose signature merges go through a `combine` callable
(the GPU's batched G1 add, `Engine.combine_g1`). Bitsets are Python ints
(bit i = registry slot min + i of the level), so Or/And/Xor/Cardinality are
single big-int operations.

Verdicts are a pure function of (msg, level range, bitset, sig): batching
changes which signatures are checked together, never a verdict.
"""

from __future__ import annotations

import queue
import threading
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import partitioner as part

# ---------------------------------------------------------------------------
# bitsets (willf semantics on Python ints)


def bits_to_int(bits: Sequence[bool]) -> int:
    v = 0
    for i, b in enumerate(bits):
        if b:
            v |= 1 << i
    return v


def int_to_bits(v: int, n: int) -> List[bool]:
    return [bool((v >> i) & 1) for i in range(n)]


def int_to_words(v: int, n: int) -> np.ndarray:
    """willf words of an n-bit set: bit i = word[i >> 6] bit (i & 63)."""
    nw = (n + 63) // 64
    return np.frombuffer(v.to_bytes(8 * nw, "little"), dtype="<u8").astype(np.uint64)


@dataclass
class MultiSig:
    """crypto.go:59-63 MultiSignature: a bitset of `bitlen` bits and a
    marshalled G1 signature (64 bytes)."""
    bitlen: int
    bits: int
    sig: bytes

    def cardinality(self) -> int:
        return self.bits.bit_count()

    def bool_list(self) -> List[bool]:
        return int_to_bits(self.bits, self.bitlen)


@dataclass(eq=False)
class IncomingSig:
    """processing.go:14-30 incomingSig. `ms` None is a packet without a
    multisignature (skipped by readTodos, processing.go:193-195)."""
    origin: int
    level: int
    ms: Optional[MultiSig]
    ind: bool = False
    mapped_index: int = 0

    def individual(self) -> bool:
        return self.ind


# processing.go:120 deathPillPair = incomingSig{origin: -1}
DEATH_PILL = IncomingSig(origin=-1, level=0, ms=None)
# the reference closes its out channel at the death pill (processing.go:254-256)
CLOSED = None


# ---------------------------------------------------------------------------
# evaluators (processing.go:32-75)


class Evaluator1:
    """processing.go:44-55: every signature gets mark 1 (verify everything)."""

    def evaluate(self, sp: IncomingSig) -> int:
        return 1


class EvaluatorStore:
    """processing.go:57-70: the store's own scoring."""

    def __init__(self, store: "Store"):
        self.store = store

    def evaluate(self, sp: IncomingSig) -> int:
        return self.store.evaluate(sp)


# ---------------------------------------------------------------------------
# filters (processing.go:290-338)


class IndividualSigFilter:
    """Accepts each origin's individual signature once (processing.go:299-325)."""

    def __init__(self):
        self.seen: Dict[int, bool] = {}

    def accept(self, inc: IncomingSig) -> bool:
        if not inc.individual():
            return True
        if inc.origin in self.seen:
            return False
        self.seen[inc.origin] = True
        return True


class CombinedFilter:
    """processing.go:327-338: the first refusing filter wins."""

    def __init__(self, filters):
        self.filters = list(filters)

    def accept(self, inc: IncomingSig) -> bool:
        return all(f.accept(inc) for f in self.filters)


# ---------------------------------------------------------------------------
# replace store (store.go)


class Store:
    """store.go:39-80 `store` for one node: best multisignature per level and
    the verified individual signatures. `combine(a, b)` returns the marshalled
    G1 sum of two marshalled signatures (SigBLS.Combine, bn256/go:192-200)."""

    def __init__(self, node_id: int, n: int, combine: Callable[[bytes, bytes], bytes]):
        self.node_id, self.n, self.combine = node_id, n, combine
        self.lock = threading.Lock()
        self.m: Dict[int, MultiSig] = {}
        self.highest = 0
        self.levels = [lvl for lvl, _, _ in part.level_sizes(node_id, n)]
        self.indiv_verified: Dict[int, int] = {0: 0}
        self.indiv_sigs: Dict[int, Dict[int, MultiSig]] = {0: {}}
        for lvl in self.levels:
            self.indiv_verified[lvl] = 0
            self.indiv_sigs[lvl] = {}

    def size(self, level: int) -> int:
        """binomialPartitioner.Size (partitioner.go:213-222): 0 for an empty level."""
        try:
            lo, hi = part.range_level(self.node_id, self.n, level)
        except part.PartitionerError as e:
            if str(e) == "empty level":
                return 0
            raise
        return hi - lo

    def evaluate(self, sp: IncomingSig) -> int:
        with self.lock:
            score = self._unsafe_evaluate(sp)
        if score < 0:
            raise AssertionError("can't have a negative score!")
        return score

    def _unsafe_evaluate(self, sp: IncomingSig) -> int:
        """store.go:111-183 unsafeEvaluate."""
        to_receive = self.size(sp.level)
        cur = self.m.get(sp.level)
        if cur is not None and to_receive == cur.cardinality():
            return 0  # completed level
        ivs = self.indiv_verified.get(sp.level, 0)
        if sp.individual() and (ivs >> sp.mapped_index) & 1:
            return 0  # individual signature already verified
        if cur is not None and not sp.individual() and (sp.ms.bits & ~cur.bits) == 0:
            return 0  # current best is a superset
        with_indiv = sp.ms.bits | ivs
        if cur is None:
            new_total = with_indiv.bit_count()
            added = new_total
            combine_ct = new_total - sp.ms.cardinality()
        elif sp.ms.bits & cur.bits:
            # overlap: replace
            new_total = with_indiv.bit_count()
            added = new_total - cur.cardinality()
            combine_ct = new_total - sp.ms.cardinality()
        else:
            final = with_indiv | cur.bits
            new_total = final.bit_count()
            added = new_total - cur.cardinality()
            combine_ct = (final ^ (cur.bits | sp.ms.bits)).bit_count()
        if added <= 0:
            return 1 if sp.individual() else 0
        if new_total == to_receive:
            return 1000000 - sp.level * 10 - combine_ct
        return 100000 - sp.level * 100 + added * 10 - combine_ct

    def store(self, sp: IncomingSig) -> Optional[MultiSig]:
        """store.go:82-99 Store: record an individual signature, then merge or
        replace the level's best (unsafeCheckMerge, store.go:185-226)."""
        with self.lock:
            if sp.individual():
                if sp.ms.cardinality() != 1:
                    raise AssertionError("bad individual sig")
                self.indiv_verified[sp.level] = self.indiv_verified.get(sp.level, 0) | (1 << sp.mapped_index)
                self.indiv_sigs.setdefault(sp.level, {})[sp.mapped_index] = sp.ms
            ms, keep = self._unsafe_check_merge(sp)
            if keep:
                self.m[sp.level] = ms
                self.highest = max(self.highest, sp.level)
            return ms

    def _unsafe_check_merge(self, sp: IncomingSig) -> Tuple[Optional[MultiSig], bool]:
        ms2 = self.m.get(sp.level)
        if ms2 is None:
            return sp.ms, True
        best = MultiSig(sp.ms.bitlen, sp.ms.bits, sp.ms.sig)
        merged = sp.ms.bits | ms2.bits
        if merged.bit_count() == ms2.cardinality() + sp.ms.cardinality():
            best = MultiSig(sp.ms.bitlen, merged, self.combine(ms2.sig, sp.ms.sig))
        vl = self.indiv_verified.get(sp.level, 0)
        i_s = (best.bits & vl) ^ vl
        if i_s.bit_count() + best.cardinality() <= ms2.cardinality():
            return None, False
        pos = 0
        while i_s >> pos:
            if (i_s >> pos) & 1:
                sig = self.indiv_sigs[sp.level].get(pos)
                if sig is None:
                    raise AssertionError("we should have this signature in our map")
                if sig.cardinality() != 1:
                    raise AssertionError("bad individual sig")
                best.bits |= 1 << pos
                best.sig = self.combine(sig.sig, best.sig)
            pos += 1
        return best, True

    def best(self, level: int) -> Tuple[Optional[MultiSig], bool]:
        with self.lock:
            ms = self.m.get(level)
            return ms, ms is not None


# ---------------------------------------------------------------------------
# batched evaluator processing (processing.go:91-287)

VerifyFn = Callable[[Sequence[IncomingSig]], List[Optional[str]]]


class BatchedEvaluatorProcessing:
    """signatureProcessing (processing.go:77-89) with a K-slot readTodos.

    `verify(sigs)` returns, per signature, None (valid) or the error text the
    reference's verifySignature would return. `log(kind, value)` receives the
    reference's Warn("verify", err) and Info("processed_sig", n) events.
    """

    def __init__(self, verify: VerifyFn, evaluator, batch: int = 64, sig_sleep_time_ms: int = 0,
                 log: Optional[Callable[[str, object], None]] = None, out_capacity: int = 1000):
        if batch < 1:
            raise ValueError("batch must be >= 1")
        self.verify, self.evaluator, self.batch = verify, evaluator, batch
        self.sig_sleep_time_ms = sig_sleep_time_ms
        self.log = log or (lambda kind, value: None)
        self.cond = threading.Condition()
        self.todos: List[IncomingSig] = []
        self.filter = IndividualSigFilter()
        self.out: "queue.Queue[Optional[IncomingSig]]" = queue.Queue(out_capacity)
        self.thread: Optional[threading.Thread] = None
        # processing.go:106-118 statistics
        self.sig_checked_ct = 0
        self.sig_queue_size = 0
        self.sig_suppressed = 0
        self.sig_checking_time = 0
        self.batches = 0

    # -- signatureProcessing interface ------------------------------------
    def start(self):
        self.thread = threading.Thread(target=self.process_loop, daemon=True)
        self.thread.start()

    def stop(self):
        self.add(DEATH_PILL)
        if self.thread is not None and self.thread is not threading.current_thread():
            self.thread.join()

    def verified(self) -> "queue.Queue[Optional[IncomingSig]]":
        return self.out

    def add(self, sp: IncomingSig):
        with self.cond:
            if self.filter.accept(sp):
                self.todos.append(sp)
                self.cond.notify()

    # -- selection ---------------------------------------------------------
    def read_todos(self) -> Tuple[bool, List[IncomingSig]]:
        """processing.go:171-220 with `batch` best slots. Each todo is scored
        once; a todo that does not beat the weakest slot (or mark 0) goes back
        to the queue in visiting order, an evicted slot is re-queued at the
        moment it is evicted — for batch = 1 exactly the reference's loop."""
        with self.cond:
            while not self.todos:
                self.cond.wait()
            previous_len = len(self.todos)
            new_todos: List[IncomingSig] = []
            slots: List[Tuple[int, IncomingSig]] = []  # descending mark, stable
            for pair in self.todos:
                if pair is DEATH_PILL or pair.origin == -1 and pair.ms is None:
                    return True, []
                if pair.ms is None:
                    continue
                mark = self.evaluator.evaluate(pair)
                if mark <= 0:
                    continue
                if len(slots) == self.batch and mark <= slots[-1][0]:
                    new_todos.append(pair)
                    continue
                if len(slots) == self.batch:
                    new_todos.append(slots.pop()[1])
                k = len(slots)
                while k > 0 and slots[k - 1][0] < mark:
                    k -= 1
                slots.insert(k, (mark, pair))
            self.todos = new_todos
            new_len = len(new_todos)
            best = [p for _, p in slots]
            self.sig_suppressed += previous_len - new_len - len(best)
            self.sig_checked_ct += len(best)
            self.sig_queue_size += new_len * len(best)
            return False, best

    # -- processing loop ---------------------------------------------------
    def process_step(self) -> bool:
        done, best = self.read_todos()
        if done:
            self.out.put(CLOSED)
            return True
        if best:
            self.verify_and_publish(best)
        return False

    def process_loop(self):
        count = 0
        while not self.process_step():
            count += 1
            if count % 100 == 0:
                self.log("processed_sig", count)

    def verify_and_publish(self, sps: Sequence[IncomingSig]):
        """processing.go:270-287 for a batch: one GPU launch, then publish the
        valid signatures in selection order and log the invalid ones."""
        t0 = time.monotonic()
        if self.sig_sleep_time_ms <= 0:
            errs = self.verify(sps)
        else:
            time.sleep(self.sig_sleep_time_ms * len(sps) / 1000.0)
            errs = [None] * len(sps)
        self.sig_checking_time += int((time.monotonic() - t0) * 1000)
        self.batches += 1
        for sp, err in zip(sps, errs):
            if err is not None:
                self.log("verify", err)
            else:
                self.out.put(sp)

    def values(self) -> Dict[str, float]:
        """processing.go:237-252 Values (means per checked signature)."""
        q = t = 0.0
        if self.sig_checked_ct > 0:
            q = self.sig_queue_size / self.sig_checked_ct
            t = self.sig_checking_time / self.sig_checked_ct
        return {"sigCheckedCt": float(self.sig_checked_ct), "sigQueueSize": q,
                "sigSuppressed": float(self.sig_suppressed), "sigCheckingTime": t,
                "sigBatches": float(self.batches)}


# ---------------------------------------------------------------------------
# several Handel instances on one GPU context (simul/node/main.go:63-131)


NodesVerifyFn = Callable[[Sequence[Tuple[int, IncomingSig]]], List[Optional[str]]]


@dataclass
class _Job:
    items: List[Tuple[int, IncomingSig]]
    done: threading.Event = field(default_factory=threading.Event)
    result: Optional[List[Optional[str]]] = None
    error: Optional[BaseException] = None


class SharedBatcher:
    """Process-wide batcher (SURVEY.md §8(b) option 1) for the k Handel
    instances one simul process runs (simul/node/main.go:63-131): each
    instance's processing calls `verify(node_id, sigs)` concurrently; a worker
    merges every pending request into ONE `target` call (normally
    `BatchVerifier.verify_nodes`, one GPU launch over the shared registry),
    flushing once `max_batch` signatures are pending or `max_wait_us` has
    passed since the worker woke. Each caller blocks until its verdicts are back."""

    def __init__(self, target: NodesVerifyFn, max_batch: int = 4096, max_wait_us: int = 200):
        self.target = target
        self.max_batch, self.max_wait = max_batch, max_wait_us / 1e6
        self.cond = threading.Condition()
        self.pending: List[_Job] = []
        self.closed = False
        self.launches = 0
        self.worker = threading.Thread(target=self._run, daemon=True)
        self.worker.start()

    def verify(self, node_id: int, sigs: Sequence[IncomingSig]) -> List[Optional[str]]:
        job = _Job([(node_id, s) for s in sigs])
        with self.cond:
            if self.closed:
                raise RuntimeError("batcher closed")
            self.pending.append(job)
            self.cond.notify_all()
        job.done.wait()
        if job.error is not None:
            raise job.error
        return job.result

    def bind(self, node_id: int) -> VerifyFn:
        """The VerifyFn of node `node_id`'s BatchedEvaluatorProcessing."""
        return lambda sigs: self.verify(node_id, sigs)

    def close(self):
        with self.cond:
            self.closed = True
            self.cond.notify_all()
        self.worker.join()

    def _npending(self) -> int:
        return sum(len(j.items) for j in self.pending)

    def _take(self) -> List[_Job]:
        with self.cond:
            while not self.pending and not self.closed:
                self.cond.wait()
            if not self.pending:
                return []
            t_end = time.monotonic() + self.max_wait
            while not self.closed and self._npending() < self.max_batch:
                left = t_end - time.monotonic()
                if left <= 0:
                    break
                self.cond.wait(left)
            take, n = [], 0
            while self.pending and (n == 0 or n + len(self.pending[0].items) <= self.max_batch):
                j = self.pending.pop(0)
                take.append(j)
                n += len(j.items)
            return take

    def _run(self):
        while True:
            jobs = self._take()
            if not jobs:
                return
            flat = [it for j in jobs for it in j.items]
            try:
                res = self.target(flat)
                self.launches += 1
                k = 0
                for j in jobs:
                    j.result = list(res[k:k + len(j.items)])
                    k += len(j.items)
            except BaseException as e:  # surfaced to every waiting caller
                for j in jobs:
                    j.error = e
            for j in jobs:
                j.done.set()
