"""GPU suite: the GT path of aggregate verification (handel_amd/csrc/bn256_gt.hip).

hg_verify_aggregate checks e(H, sum of set keys) == e(sig, G2Base) as
FE(Miller(G2Base at -sig)) == conj(prod of per-key GT values), with the
per-key values e(H, pk_i) and their window/block products built once per
(message, registry). These tests pin the table life cycle (message and
registry changes, hg_prepare_aggregate) and the GT verdicts against the C
restatement of the reference (oracle/bn256_ref.c) and against the G2 point
fold (HG_AGG_PATH=g2, run in a child process).
"""

import json
import os
import subprocess
import sys

import numpy as np
import pytest

from handel_amd._lib import HG_ERR_HASH_EOF, HandelGPUError
from handel_amd.engine import REQ_DTYPE, Engine
from oracle import bn256_oracle as O
from oracle import ref_lib as R
from tests import _fixtures as F

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _batch(ks, reg_n, msg, ranges, rng, tamper_every=5):
    """Aggregate signatures of random bitsets over the given ranges, signed on msg."""
    bitsets = F.random_bitsets(rng, [s for _, s in ranges])
    for b in bitsets:
        b[int(rng.integers(len(b)))] = True
    h = O.hashed_message(msg)[0]
    sigs = bytearray()
    for (off, _), bits in zip(ranges, bitsets):
        k = sum(ks[off + i] for i, b in enumerate(bits) if b) % O.ORDER
        sigs += O.g1_marshal(O.g1_mul(h, k))
    sigs = F.tamper(bytes(sigs), every=tamper_every)
    reqs, words = F.pack_requests(ranges, bitsets)
    return np.array(reqs, dtype=REQ_DTYPE), words, sigs


def _levels(n_reg, nodes):
    out = []
    for node in nodes:
        for lvl in range(1, O.log2_ceil(n_reg) + 1):
            rl, err = O.range_level(node, n_reg, lvl)
            if err is None:
                out.append((rl[0], rl[1] - rl[0]))
    return sorted(set(out)) + [(0, n_reg)]


def _oracle(msg, reg, reqs, words, sigs):
    return R.verify_aggregate(msg, reg, reqs["offset"], reqs["bitlen"], reqs["level_size"], words,
                              reqs["word_offset"].astype(np.uint64), sigs, nthreads=8)


def test_prepare_aggregate_states(engine):
    """hg_prepare_aggregate: needs a message and a registry; a hash-rejected
    message has nothing to build; otherwise builds (and then reuses) the tables."""
    ks = F.scalars(20, seed=b"gt-prep")
    reg = R.g2_scalar_base(F.scalar_bytes(ks))
    assert list(engine.registry_load(reg)) == [0] * 20
    assert engine.set_message(F.REJECT_MESSAGES[0]) == HG_ERR_HASH_EOF
    assert engine.prepare_aggregate() == HG_ERR_HASH_EOF
    assert engine.set_message(F.LIB_MESSAGE) == 0
    assert engine.prepare_aggregate() == 0
    assert engine.prepare_aggregate() == 0  # cached


def test_prepare_aggregate_without_registry(engine_cf):
    """A context whose registry failed to load has no registry: HG_ERR_ARG."""
    bad = bytes([0xff]) * 128
    engine_cf.registry_load(bad)
    assert engine_cf.set_message(F.LIB_MESSAGE) == 0
    with pytest.raises(HandelGPUError, match="hg_prepare_aggregate"):
        engine_cf.prepare_aggregate()


def test_tables_follow_message_and_registry(engine):
    """The tables are e(H, .) of the CURRENT message and registry: switching
    either rebuilds them, so signatures verify exactly under their own
    message / registry (and a message's signatures fail under another)."""
    rng = np.random.default_rng(3)
    msgs = [F.LIB_MESSAGE, F.TEST_MESSAGES[0]]
    regs = []
    for seed in (b"gt-regA", b"gt-regB"):
        ks = F.scalars(96, seed=seed)
        regs.append((ks, R.g2_scalar_base(F.scalar_bytes(ks))))
    ranges = _levels(96, (0, 41, 95))
    for ri, (ks, reg) in enumerate(regs):
        assert list(engine.registry_load(reg)) == [0] * 96
        for mi, msg in enumerate(msgs):
            reqs, words, sigs = _batch(ks, 96, msg, ranges, rng)
            for use in msgs:  # the same signatures under both messages
                codes = engine.verify_aggregate_msg(use, reqs, words, sigs)
                want = _oracle(use, reg, reqs, words, sigs)
                assert list(codes) == list(want), (ri, mi, use)
                if use == msg:
                    assert (np.asarray(codes) == 0).sum() > len(ranges) // 2
                else:
                    assert (np.asarray(codes) == 0).sum() == 0


def test_two_messages_keep_their_tables():
    """Interleaved messages on ONE context: the context
    caches the current and the previous message's hashedMessage and GT tables
    (bn256/go/bn256.go:210-218: H, and every table, is fixed per message), so
    alternating two messages stays at table level 2 with the oracle's
    verdicts, and a table budget that holds one message's tables only drops
    the other's."""
    e = Engine(device=0, flavor="go")
    try:
        rng = np.random.default_rng(11)
        ks = F.scalars(64, seed=b"two-msgs")
        reg = R.g2_scalar_base(F.scalar_bytes(ks))
        assert list(e.registry_load(reg)) == [0] * 64
        msgs = [F.LIB_MESSAGE, F.TEST_MESSAGES[1]]
        ranges = _levels(64, (3, 40))
        batches = [_batch(ks, 64, m, ranges, rng) for m in msgs]
        wants = [_oracle(m, reg, *b) for m, b in zip(msgs, batches)]
        for m in msgs:
            assert e.prepare_aggregate_msg(m) == 0
        for i in range(6):
            k = i % 2
            codes = e.verify_aggregate_msg(msgs[k], *batches[k])
            assert list(codes) == list(wants[k]), i
            assert e.aggregate_tables() == 2, i
        both = e.context_bytes()
        # a budget for one message's level-2 tables: the cached message's go first
        one = 64 // 16 * 65536 * 480 + 64 * 480 * 300
        e.set_table_budget(one)
        assert e.context_bytes() < both
        assert e.aggregate_tables() == 2
        codes = e.verify_aggregate_msg(msgs[1], *batches[1])
        assert list(codes) == list(wants[1])
    finally:
        e.close()


_CHILD = r"""
import json, os, sys
import numpy as np
sys.path.insert(0, %r)
import bench
from handel_amd.engine import Engine
e = Engine(device=0, flavor="go")
assert e.set_message(bench.LIB_MESSAGE) == 0
reqs, words, sigs, expect, _, reg = bench.make_aggregate_batch(e, 1000, 1024, seed=5)
codes = e.verify_aggregate(reqs, words, sigs)
print(json.dumps({"codes": [int(c) for c in codes], "level": e.aggregate_tables()}))
""" % ROOT


def _child(env_over, code=_CHILD):
    env = {k: v for k, v in os.environ.items() if k not in ("HG_GT_LEVEL", "HG_AGG_PATH", "HG_SIG12", "HG_SIG_W2")}
    env.update(env_over)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_gt_and_g2_paths_agree():
    """Every table level gives the oracle's verdicts on the same batch (1024
    multisigs at random Handel levels of a 1000-key registry): the GT fold over
    16-key windows (HG_GT_LEVEL=2), over 8-key windows (1), the G2 point fold
    + two-pairing check (0, and HG_AGG_PATH=g2) — each in a child process."""
    outs = {}
    # gt16c16 / gt16c5: chunks of 16 and 5 terms per fold team (HG_GT_CHUNK):
    # a 12-lane team (k_gt_chunks) reads terms past 12 from the term list
    runs = (("gt16", {"HG_GT_LEVEL": "2"}), ("gt8", {"HG_GT_LEVEL": "1"}),
            ("g2", {"HG_GT_LEVEL": "0"}), ("g2env", {"HG_AGG_PATH": "g2"}),
            ("gt16c16", {"HG_GT_LEVEL": "2", "HG_GT_CHUNK": "16"}),
            ("gt16c5", {"HG_GT_LEVEL": "2", "HG_GT_CHUNK": "5"}),
            # the signature pairing on 12-lane teams (bn256_sig12.hip) on the
            # padded context path too, and the 16-lane kernel everywhere (the
            # 1024-check batch: two-wave teams, k_verify_sig_split<2>, unless
            # HG_SIG_W2=0)
            ("gt16sig12", {"HG_GT_LEVEL": "2", "HG_SIG12": "1"}),
            ("gt16sig16", {"HG_GT_LEVEL": "2", "HG_SIG12": "0"}),
            ("gt16w1", {"HG_GT_LEVEL": "2", "HG_SIG12": "0", "HG_SIG_W2": "0"}))
    for name, env in runs:
        outs[name] = _child(env)
    assert [outs[k]["level"] for k, _ in runs] == [2, 1, 0, 0, 2, 2, 2, 2, 2]
    assert all(outs[k]["codes"] == outs["gt16"]["codes"] for k, _ in runs)
    import bench
    from handel_amd.engine import Engine

    e = Engine(device=0, flavor="go")
    try:
        assert e.set_message(bench.LIB_MESSAGE) == 0
        reqs, words, sigs, expect, _, reg = bench.make_aggregate_batch(e, 1000, 1024, seed=5)
    finally:
        e.close()
    assert outs["gt16"]["codes"] == [int(c) for c in expect]
    assert outs["gt16"]["codes"] == [int(c) for c in _oracle(bench.LIB_MESSAGE, reg, reqs, words, sigs)]


def test_volume_policy():
    """Without HG_GT_LEVEL: a message's first requests use the G2 fold, the
    8-key GT tables appear once 16384 requests have come in, a switch to
    another message and back keeps them (the context caches two messages),
    a third message evicts them, hg_prepare_aggregate builds the 16-key level
    — and the verdicts are the same at every step."""
    code = r"""
import json, sys
import numpy as np
sys.path.insert(0, %r)
import bench
from handel_amd.engine import Engine
e = Engine(device=0, flavor="go")
assert e.set_message(bench.LIB_MESSAGE) == 0
reqs, words, sigs, expect, _, reg = bench.make_aggregate_batch(e, 500, 3000, seed=9)
out = []
def run(a, b):
    c = e.verify_aggregate(reqs[a:b], words, sigs[64 * a:64 * b])
    out.append((bool(np.array_equal(c, expect[a:b])), e.aggregate_tables()))
run(0, 1000)
for _ in range(5):
    run(0, 3000)         # 16000 requests so far: still the G2 fold
run(1000, 2000)          # 17000: the 8-key tables
assert e.set_message(b"Peaches and Cream") == 0
assert e.set_message(bench.LIB_MESSAGE) == 0
run(0, 100)              # the previous message's tables are kept
assert e.set_message(b"Peaches and Cream") == 0
assert e.set_message(b"Get Funky Tonight") == 0
assert e.set_message(bench.LIB_MESSAGE) == 0
run(0, 100)              # two other messages since: evicted
assert e.prepare_aggregate() == 0
run(0, 3000)
print(json.dumps(out))
""" % ROOT
    env = {k: v for k, v in os.environ.items() if k not in ("HG_GT_LEVEL", "HG_AGG_PATH")}
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert [ok for ok, _ in out] == [True] * 10
    assert [lvl for _, lvl in out] == [0] * 6 + [1, 1, 0, 2]


def test_sig_edge_cases_on_gt_path(engine):
    """Signature-side edge cases through the GT check: infinity signature
    (valid only for an aggregate key at infinity), off-curve signature
    (decode error), and a duplicated key folded twice."""
    n = 64
    ks = F.scalars(n, seed=b"gt-edge")
    ks[9] = ks[8]
    reg = bytearray(R.g2_scalar_base(F.scalar_bytes(ks)))
    reg[128 * 20:128 * 21] = bytes(128)  # a registry key at infinity
    reg = bytes(reg)
    assert list(engine.registry_load(reg)) == [0] * n
    msg = F.LIB_MESSAGE
    assert engine.set_message(msg) == 0
    h = O.hashed_message(msg)[0]
    cases = [  # (offset, size, set bits, signature)
        (8, 8, [0, 1], None),          # keys 8 and 9 are equal: 2 k8 H
        (16, 8, [4], "inf"),           # only the infinity key: aggregate = infinity
        (16, 8, [4], None),            # ... with the honest signature (also infinity)
        (16, 8, [3, 4], None),         # infinity key beside a real one
        (0, 64, list(range(64)), None),
        (32, 32, list(range(32)), "offcurve"),
        (0, 8, [1], "inf"),            # infinity signature on a real key: invalid
    ]
    ranges, bitsets, sigs = [], [], bytearray()
    for off, size, bits, kind in cases:
        ranges.append((off, size))
        b = [False] * size
        for i in bits:
            b[i] = True
        bitsets.append(b)
        k = sum(0 if off + i == 20 else ks[off + i] for i in bits) % O.ORDER
        if kind == "inf":
            sigs += bytes(64)
        elif kind == "offcurve":
            sigs += (1).to_bytes(32, "big") + (1).to_bytes(32, "big")
        else:
            sigs += O.g1_marshal(O.g1_mul(h, k)) if k else bytes(64)
    reqs, words = F.pack_requests(ranges, bitsets)
    reqs = np.array(reqs, dtype=REQ_DTYPE)
    codes = engine.verify_aggregate(reqs, words, bytes(sigs))
    want = _oracle(msg, reg, reqs, words, bytes(sigs))
    assert list(codes) == list(want)
    assert list(codes[:5]) == [0, 0, 0, 0, 0] and codes[6] == 1


@pytest.mark.parametrize("n_reg", [1, 2, 15, 17, 33, 100])
def test_gt_small_and_ragged_registries(engine, n_reg):
    """Registries that end inside a 16-key window (absent keys are 1 in the
    window table) and inside a block (clipped top blocks), down to a single
    key: every Handel level range of several nodes, plus level errors."""
    rng = np.random.default_rng(n_reg)
    ks = F.scalars(n_reg, seed=b"gt-small-%d" % n_reg)
    reg = R.g2_scalar_base(F.scalar_bytes(ks))
    assert list(engine.registry_load(reg)) == [0] * n_reg
    msg = F.TEST_MESSAGES[1]
    assert engine.set_message(msg) == 0
    nodes = sorted({0, n_reg - 1, n_reg // 2})
    ranges = _levels(n_reg, nodes) if n_reg > 1 else [(0, 1)]
    reqs, words, sigs = _batch(ks, n_reg, msg, ranges, rng, tamper_every=3)
    # one request past the registry end and one with bitlen != level size
    bad = np.array([(max(0, n_reg - 1), 2, 2, 0), (0, 1, 2, 0)], dtype=REQ_DTYPE)
    reqs = np.concatenate([reqs, bad])
    sigs = sigs + sigs[:64] * 2
    codes = engine.verify_aggregate(reqs, words, sigs)
    assert list(codes) == list(_oracle(msg, reg, reqs, words, sigs))
    assert list(codes[-2:]) == [3, 3]


def test_registry_above_16key_limit_uses_8key_tables(engine):
    """Registries above 16384 keys (16-key tables > 32 GB) stop at the 8-key
    GT tables: hg_prepare_aggregate builds level 1, and verdicts over the
    ragged last window (key 16384) and a full half match the oracle."""
    import bench

    n_reg = 16385
    kb = bench.seeded_scalars(n_reg, 99)
    reg = engine.keygen(kb)
    assert not engine.registry_load(reg).any()
    assert engine.set_message(F.LIB_MESSAGE) == 0
    assert engine.prepare_aggregate() == 0
    assert engine.aggregate_tables() == 1
    scal = [int.from_bytes(kb[32 * i:32 * i + 32], "big") for i in range(n_reg)]
    ranges = [(16376, 9), (0, 16), (8192, 8192), (16384, 1)]
    rng = np.random.default_rng(8)
    reqs, words, sigs = _batch(scal, n_reg, F.LIB_MESSAGE, ranges, rng, tamper_every=2)
    codes = engine.verify_aggregate(reqs, words, sigs)
    assert list(codes) == list(_oracle(F.LIB_MESSAGE, reg, reqs, words, sigs))
    assert list(codes) == [1, 0, 1, 0]


def test_error_precedence_on_gt_path(engine):
    """Verdict precedence of the GT path's prologue kernel (k_agg_prologue +
    k_gt_plan), through the host and the device entry points: signature decode
    error (the packet parse, before processing) > level error
    (processing.go:350-352) > empty bitset (the nil-aggregate panic) > pairing
    verdict. Single-error rows are also checked against the oracle."""
    import torch

    n = 32
    ks = F.scalars(n, seed=b"gt-prec")
    reg = R.g2_scalar_base(F.scalar_bytes(ks))
    assert list(engine.registry_load(reg)) == [0] * n
    msg = F.LIB_MESSAGE
    assert engine.set_message(msg) == 0
    assert engine.prepare_aggregate() == 0
    h = O.hashed_message(msg)[0]
    off_curve = (1).to_bytes(32, "big") + (1).to_bytes(32, "big")

    def honest(off, bits):
        k = sum(ks[off + i] for i, b in enumerate(bits) if b and off + i < n) % O.ORDER
        return O.g1_marshal(O.g1_mul(h, k))

    rows = [  # (offset, level size, bits, signature, expected code)
        (0, 8, [True, True] + [False] * 6, None, 0),
        (8, 16, [True] * 8, off_curve, 5),        # bad signature beats the level error
        (8, 16, [False] * 8, None, 3),            # level error beats the empty bitset
        (16, 8, [False] * 8, None, 6),            # empty bitset: nil aggregate
        (16, 8, [False] * 8, off_curve, 5),       # bad signature beats the empty bitset
        (24, 16, [True] * 16, None, 3),           # range past the registry
        (0, 16, [True] * 16, "tamper", 1),        # pairing verdict
    ]
    ranges, bitsets, sigs = [], [], bytearray()
    for off, size, bits, sig, _ in rows:
        ranges.append((off, size))
        bitsets.append(bits)
        if sig is None:
            sigs += honest(off, bits) if any(bits) else honest(0, [True])
        elif sig == "tamper":
            s = honest(off, bits)
            sigs += O.g1_marshal(O.g1_add(O.g1_unmarshal(s)[0], O.g1_unmarshal(honest(0, [True]))[0]))
        else:
            sigs += sig
    reqs, words = F.pack_requests(ranges, bitsets)
    reqs = np.array(reqs, dtype=REQ_DTYPE)
    want = [code for *_, code in rows]
    assert list(engine.verify_aggregate(reqs, words, bytes(sigs))) == want
    single = [0, 2, 3, 5, 6]  # rows with at most one error: the oracle agrees
    oracle = _oracle(msg, reg, reqs, words, bytes(sigs))
    assert [int(oracle[i]) for i in single] == [want[i] for i in single]
    dev = torch.device("cuda", 0)
    d_reqs = torch.frombuffer(bytearray(reqs.tobytes()), dtype=torch.uint8).to(dev)
    d_words = torch.frombuffer(bytearray(words.tobytes()), dtype=torch.uint8).to(dev)
    d_sigs = torch.frombuffer(bytearray(sigs), dtype=torch.uint8).to(dev)
    d_codes = torch.full((len(rows),), -1, dtype=torch.int32, device=dev)
    engine.verify_aggregate_device(d_reqs.data_ptr(), len(rows), d_words.data_ptr(), d_sigs.data_ptr(),
                                   d_codes.data_ptr(), 0, torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize(dev)
    assert d_codes.cpu().tolist() == want


@pytest.mark.parametrize("seed,n_reg,m", [(1, 37, 1), (2, 100, 7), (3, 257, 64), (4, 1000, 300), (5, 1000, 777),
                                          (6, 4000, 129)])
def test_random_batches_match_oracle(engine, seed, n_reg, m):
    """Randomised GT-path batches against the oracle: random registry sizes,
    random nodes and Handel levels (partitioner rangeLevel), bitset densities
    from empty to full (so plain, complemented and empty folds all occur),
    every 5th aggregate tampered."""
    rng = np.random.default_rng(seed)
    ks = F.scalars(n_reg, seed=b"gt-rand-%d" % seed)
    reg = engine.keygen(F.scalar_bytes(ks))
    assert not engine.registry_load(reg).any()
    msg = F.LIB_MESSAGE
    assert engine.set_message(msg) == 0
    assert engine.prepare_aggregate() == 0
    levels = _levels(n_reg, [int(x) for x in rng.integers(0, n_reg, size=8)])
    ranges = [levels[int(i)] for i in rng.integers(0, len(levels), size=m)]
    bitsets = []
    for _, size in ranges:
        d = float(rng.choice([0.0, 0.02, rng.uniform(0.5, 1.0), 0.97, 1.0]))
        bitsets.append([bool(b) for b in rng.random(size) < d])
    scal = bytearray()
    for (off, _), bits in zip(ranges, bitsets):
        k = sum(ks[off + i] for i, b in enumerate(bits) if b) % O.ORDER
        scal += (k if k else 1).to_bytes(32, "big")
    sigs = F.tamper(engine.sign(bytes(scal)), every=5)
    reqs, words = F.pack_requests(ranges, bitsets)
    reqs = np.array(reqs, dtype=REQ_DTYPE)
    got = engine.verify_aggregate(reqs, words, sigs)
    want = _oracle(msg, reg, reqs, words, sigs)
    assert list(got) == list(want)
    assert (got == 0).any() or m < 8


def test_policy_switches_on_the_crossing_batch():
    """Device-stream order of the volume policy: the batch that takes a
    message past 16384 requests builds the 8-key tables inside its own
    submission and already runs on them; every batch's verdicts are the
    expected ones, before and after."""
    code = r"""
import json, sys
import numpy as np
sys.path.insert(0, %r)
import bench
from handel_amd.engine import Engine
e = Engine(device=0, flavor="go")
assert e.set_message(bench.LIB_MESSAGE) == 0
reqs, words, sigs, expect, _, reg = bench.make_aggregate_batch(e, 1000, 4096, seed=13)
levels, ok = [], []
for i in range(6):   # 24576 requests: the threshold is crossed on the 4th batch
    c = e.verify_aggregate(reqs, words, sigs)
    ok.append(bool(np.array_equal(c, expect)))
    levels.append(e.aggregate_tables())
print(json.dumps({"ok": ok, "levels": levels}))
""" % ROOT
    env = {k: v for k, v in os.environ.items() if k not in ("HG_GT_LEVEL", "HG_AGG_PATH")}
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["ok"] == [True] * 6
    assert out["levels"] == [0, 0, 0, 1, 1, 1]


@pytest.mark.parametrize("level,overlap", [(2, 1), (2, 0), (0, 1)], ids=["gt-overlap", "gt-serial", "g2fold"])
def test_fused_bitset_matches_pack(level, overlap):
    """hg_verify_aggregate_device_bits: the codes are the plain call's and the
    bitset is hg_pack_verdicts_device's, on a batch whose size is not a
    multiple of 8 (the tail byte), through the fused compare (GT path beside
    the fold), the serial GT path and the G2 fold (pack after the check)."""
    import torch

    import bench
    from handel_amd.engine import Engine

    e = Engine(device=0, flavor="go")
    try:
        assert e.set_message(bench.LIB_MESSAGE) == 0
        n = 1001
        reqs, words, sigs, expect, _, _ = bench.make_aggregate_batch(e, 700, n, seed=77)
        e.set_aggregate_level(level)
        e.set_fold_overlap(overlap)
        dev = torch.device("cuda", 0)
        d_reqs = torch.from_numpy(reqs.view(np.uint8).copy()).to(dev)
        d_words = torch.from_numpy(words.view(np.int64).copy()).to(dev)
        d_sigs = torch.from_numpy(np.frombuffer(sigs, dtype=np.uint8).copy()).to(dev)
        codes = torch.full((n,), -1, dtype=torch.int32, device=dev)
        bits = torch.full(((n + 7) // 8,), 0xAA, dtype=torch.uint8, device=dev)
        ref = torch.zeros((n + 7) // 8, dtype=torch.uint8, device=dev)
        s = torch.cuda.current_stream(dev).cuda_stream
        for _ in range(2):  # the second submission reuses every workspace
            e.verify_aggregate_device_bits(d_reqs.data_ptr(), n, d_words.data_ptr(), d_sigs.data_ptr(),
                                           codes.data_ptr(), bits.data_ptr(), s)
        e.pack_verdicts_device(codes.data_ptr(), n, ref.data_ptr(), s)
        torch.cuda.synchronize(dev)
        assert np.array_equal(codes.cpu().numpy(), expect)
        assert torch.equal(bits, ref)
        assert e.aggregate_tables() == level
    finally:
        e.close()


@pytest.mark.parametrize("pad", [False, True, "latency"], ids=["unpadded", "padded", "latency"])
def test_device_lanes_keep_batches_in_flight(pad):
    """hg_lane_submit_device (bench.py's headline): two lanes of one context
    alternate on a batch resident in HBM, each on its own torch stream, two
    batches in flight; every round's codes are the expected verdicts (the
    oracle's: test_gt_and_g2_paths_agree) and its bitset packs them.
    'latency': padded lanes in the two-wave latency form
    (hg_lane_set_latency_form, as the verifier service sets it)."""
    import torch

    import bench
    from handel_amd.distributed import pack_verdicts
    from handel_amd.engine import DeviceLane

    dev = torch.device("cuda", 0)
    e = Engine(device=0, flavor="go")
    lanes = []
    try:
        assert e.set_message(bench.LIB_MESSAGE) == 0
        reqs, words, sigs, expect, _, reg = bench.make_aggregate_batch(e, 1000, 1024, seed=5)
        assert e.prepare_aggregate() == 0
        n = len(reqs)
        d_reqs, d_words = bench._dev_bytes(reqs.tobytes(), dev), bench._dev_bytes(words.tobytes(), dev)
        d_sigs = bench._dev_bytes(bytes(sigs), dev)
        lanes = [DeviceLane(e, n, pad=pad is not False) for _ in range(2)]
        if pad == "latency":
            for ln in lanes:
                ln.set_latency_form(2048)
        streams = [torch.cuda.Stream(dev) for _ in lanes]
        codes = [torch.full((n,), -1, dtype=torch.int32, device=dev) for _ in lanes]
        bits = [torch.zeros((n + 7) // 8, dtype=torch.uint8, device=dev) for _ in lanes]
        for rnd in range(6):
            i = rnd % 2
            with torch.cuda.stream(streams[i]):
                if rnd >= 2:  # the previous round of this lane was read: rewrite the outputs
                    codes[i].fill_(-1)
                lanes[i].submit_device(d_reqs.data_ptr(), n, d_words.data_ptr(), d_sigs.data_ptr(),
                                       codes[i].data_ptr(), bits[i].data_ptr(), streams[i].cuda_stream)
                got = codes[i].cpu().numpy()  # in the stream's order: after the lane's verdicts
            assert np.array_equal(got, expect), (pad, rnd)
            assert torch.equal(bits[i], pack_verdicts(codes[i])), (pad, rnd)
        # the context's own submissions wait for the lanes' batches
        assert list(e.verify_aggregate(reqs, words, sigs)) == list(expect)
    finally:
        for ln in lanes:
            ln.close()
        e.close()
