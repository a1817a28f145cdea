"""GPU suite: the headline's exact path against the oracle.

bench.py's headline (BASELINE config 3, and config 5 with --committees) does
not run the context's padded submission: it keeps FOUR 4096-request batches
in flight on four `DeviceLane(pad=False)` lanes of one context — unpadded
lanes run the 12-lane signature pairing (k_sig_scalars + k_sig_lines +
`k_verify_sig12<false>`, hg_api.cpp sig12_for, bn256_sig12.hip), each lane
ordered on its own stream, nothing synchronised between batches (bench.py
`lane_step`). This
suite runs that path at full size and compares every lane's verdict codes and
packed bitset with the C restatement of the reference algorithm
(R.verify_aggregate: processing.go:342-368 verifySignature ->
PublicKey.Combine per set bit -> bn256/go/bn256.go:82-94 VerifySignature),
not with the construction pattern the bench checks.

The batches carry the edge codes the reference produces besides the tampered
1/8: undecodable signatures (bn256.go Unmarshal), bit lengths that disagree
with the level (processing.go:350-352) and empty bitsets (the nil-aggregate
case). Two different batches alternate over the lanes, so a lane that read
another lane's workspace would return the other batch's verdicts.
"""

import numpy as np
import pytest

from oracle import ref_lib as R
from tests import _fixtures as F

pytestmark = pytest.mark.gpu

INFLIGHT = 4
ROUNDS = 12


def _damage(reqs, words, sigs: bytes):
    """Edge requests spread over the batch: every 29th signature bytes made
    undecodable (x >= p), every 31st request's bit length off its level, every
    37th bitset emptied. Returns new (reqs, words, sigs)."""
    reqs = reqs.copy()
    words = words.copy()
    s = bytearray(sigs)
    n = len(reqs)
    for i in range(3, n, 29):
        s[64 * i:64 * i + 32] = b"\xff" * 32  # x >= p: not a field element
    for i in range(5, n, 31):
        if reqs[i]["bitlen"] > 1:
            reqs[i]["bitlen"] -= 1  # the bitset no longer spans its level
    for i in range(7, n, 37):
        nw = (int(reqs[i]["bitlen"]) + 63) // 64
        wo = int(reqs[i]["word_offset"])
        words[wo:wo + nw] = 0
    return reqs, words, bytes(s)


def _permute(reqs, words, sigs: bytes, seed: int):
    """The same requests in another order (their words stay put)."""
    p = np.random.default_rng(seed).permutation(len(reqs))
    return reqs[p].copy(), words, b"".join(sigs[64 * i:64 * i + 64] for i in p), p


CF_SIG_CODES = {"bn256: coordinate exceeds modulus": 10, "bn256: malformed point": 11,
                "bn256: not enough data": 12}  # HG_ERR_SIG_CF_* (include/handel_gpu.h)


def _oracle(reg, reqs, words, sigs, flavor: str):
    """R.verify_aggregate (the reference algorithm; x/crypto decode rules).
    The registry's honest keys decode identically under both flavors and the
    decode step's place in the precedence is the same, so for cloudflare only
    the undecodable signatures' codes change: SigBLS.UnmarshalBinary's wrapped
    cloudflare error (bn256/cf/bn256.go:183-190), from the Python oracle."""
    from oracle import bn256_oracle as O

    codes = R.verify_aggregate(F.LIB_MESSAGE, reg, reqs["offset"], reqs["bitlen"], reqs["level_size"], words,
                               reqs["word_offset"].astype(np.uint64), sigs, nthreads=16)
    if flavor == "cf":
        for i in np.flatnonzero(codes == 5):
            _, err = O.g1_unmarshal(sigs[64 * i:64 * i + 64], "cf")
            codes[i] = CF_SIG_CODES[err]
    return codes


def _run_lanes(engine, batches):
    """bench.py's lane_step over `batches` (round r -> lane r % INFLIGHT, batch
    r % len(batches)), no synchronisation until the end; returns per lane the
    (batch index, codes, bits) of its last round."""
    import torch

    import bench
    from handel_amd.engine import DeviceLane

    dev = torch.device("cuda", 0)
    n = len(batches[0][0])
    dbs = [(bench._dev_bytes(r.tobytes(), dev), bench._dev_bytes(w.tobytes(), dev), bench._dev_bytes(s, dev))
           for r, w, s in batches]
    lanes = [DeviceLane(engine, n, pad=False) for _ in range(INFLIGHT)]
    try:
        codes = [torch.full((n,), -7, dtype=torch.int32, device=dev) for _ in lanes]
        bits = [torch.full(((n + 7) // 8,), 0x5A, dtype=torch.uint8, device=dev) for _ in lanes]
        last = [None] * INFLIGHT
        for rnd in range(ROUNDS):
            i, b = rnd % INFLIGHT, rnd % len(batches)
            d_r, d_w, d_s = dbs[b]
            lanes[i].submit_device(d_r.data_ptr(), n, d_w.data_ptr(), d_s.data_ptr(), codes[i].data_ptr(),
                                   bits[i].data_ptr(), lanes[i].stream)
            last[i] = b
        torch.cuda.synchronize(dev)
        return [(last[i], codes[i].cpu().numpy(), bits[i].cpu().numpy()) for i in range(INFLIGHT)]
    finally:
        for ln in lanes:
            ln.close()


def _check(out, wants):
    for lane, (b, codes, bits) in enumerate(out):
        want = wants[b]
        bad = np.flatnonzero(codes != want)
        assert bad.size == 0, f"lane {lane} batch {b}: {bad.size} verdicts differ, first {bad[:6]} " \
                              f"got {codes[bad[:6]]} want {want[bad[:6]]}"
        n = len(want)
        assert np.array_equal(bits, np.packbits(np.concatenate([want == 0, np.zeros((-n) % 8, bool)]),
                                                bitorder="little")), f"lane {lane} bitset"


@pytest.mark.parametrize("flavor", ["go", "cf"])
def test_headline_lanes_match_oracle_config3(request, flavor):
    """Config 3 at full size (4096 multisigs, 4000-key registry, random node
    and level) through four unpadded lanes in flight, both flavors."""
    import bench

    engine = request.getfixturevalue("engine" if flavor == "go" else "engine_cf")
    assert engine.set_message(F.LIB_MESSAGE) == 0
    reqs, words, sigs, expect, _, reg = bench.make_aggregate_batch(engine, 4000, 4096, seed=4321)
    assert engine.prepare_aggregate() == 0 and engine.aggregate_tables() == 2
    a = _damage(reqs, words, sigs)
    pr, pw, ps, _ = _permute(*a, seed=2)
    wants = [_oracle(reg, *a, flavor), _oracle(reg, pr, pw, ps, flavor)]
    # the damage produced every edge code, and the tampered 1/8 still fail
    assert {0, 1, 3, 6} <= set(wants[0].tolist()) and (5 if flavor == "go" else 10) in set(wants[0].tolist())
    out = _run_lanes(engine, [a, (pr, pw, ps)])
    _check(out, wants)
    # the context's own (padded) submission agrees with the lanes
    assert np.array_equal(engine.verify_aggregate(*a), wants[0])


@pytest.mark.parametrize("flavor", ["go", "cf"])
def test_headline_lanes_match_oracle_committee(request, flavor):
    """Config 5's unit (bench.py --committees): a 4096-key committee registry,
    3584 multisigs at random levels + 512 over the whole registry, through the
    same four unpadded lanes."""
    from tests.test_gpu_committee import committee_batch

    engine = request.getfixturevalue("engine" if flavor == "go" else "engine_cf")
    assert engine.set_message(F.LIB_MESSAGE) == 0
    reqs, words, sigs, expect, reg = committee_batch(engine)
    assert engine.prepare_aggregate() == 0 and engine.aggregate_tables() == 2
    a = _damage(reqs, words, sigs)
    pr, pw, ps, _ = _permute(*a, seed=4)
    wants = [_oracle(reg, *a, flavor), _oracle(reg, pr, pw, ps, flavor)]
    out = _run_lanes(engine, [a, (pr, pw, ps)])
    _check(out, wants)


def test_pairing_kernels_give_identical_fe_values(engine, engine_cf):
    """hg_sig_pairing_device: the 16-lane k_verify_sig (padded, unpadded) and
    the 12-lane k_verify_sig12 (padded, unpadded, with k_sig_scalars /
    k_sig_lines) and the two-wave k_verify_sig_split<2> write byte-identical FE(Miller(G2Base at -sig)) values for
    valid signatures and the point at infinity, ragged n (teams of the last
    wave partly empty), both flavors. The verdict tests pin those values to
    the oracle through the comparison with the fold."""
    import torch

    import bench

    dev = torch.device("cuda", 0)
    for eng in (engine, engine_cf):
        assert eng.set_message(F.LIB_MESSAGE) == 0
        for n in (1, 7, 61, 1029):
            kb = bench.seeded_scalars(n, 900 + n)
            sigs = bytearray(eng.sign(kb))
            sigs[0:64] = bytes(64)  # the point at infinity
            d_sigs = bench._dev_bytes(bytes(sigs), dev)
            outs = []
            for k in range(5):
                fe = torch.full((n * 480,), 0x5A, dtype=torch.uint8, device=dev)
                # (torch's default stream is handle 0: the context's own stream runs it)
                eng.sig_pairing_device(d_sigs.data_ptr(), n, fe.data_ptr(), k,
                                       torch.cuda.current_stream(dev).cuda_stream)
                torch.cuda.synchronize(dev)
                outs.append(fe.cpu().numpy())
            for k in range(1, 5):
                assert np.array_equal(outs[0], outs[k]), (eng.flavor_name, n, k)
            # e(inf, G2Base) = 1: the first value is the GT identity (only
            # element 1, c0.y, nonzero: one in Montgomery form)
            v = outs[0][:480].view(np.uint32).reshape(12, 10)
            nz = [e for e in range(12) if v[e].any()]
            assert nz == [1], (eng.flavor_name, n, nz, v[:2].tolist())


_MONO_CHILD = r"""
import os, sys
sys.path.insert(0, os.environ["HG_ROOT"])
import numpy as np, torch
import bench
from handel_amd.engine import Engine
dev = torch.device("cuda", 0)
out = []
for flavor in ("go", "cf"):
    eng = Engine(device=0, flavor=flavor)
    assert eng.set_message(bench.LIB_MESSAGE) == 0
    for n in (7, 1029):
        sigs = bytearray(eng.sign(bench.seeded_scalars(n, 1900 + n)))
        sigs[64:128] = bytes(64)
        d = torch.frombuffer(bytearray(sigs), dtype=torch.uint8).to(dev)
        for k in (2, 3):
            fe = torch.full((n * 480,), 0x5A, dtype=torch.uint8, device=dev)
            eng.sig_pairing_device(d.data_ptr(), n, fe.data_ptr(), k, torch.cuda.current_stream(dev).cuda_stream)
            torch.cuda.synchronize(dev)
            out.append(fe.cpu().numpy())
    eng.close()
np.save(sys.argv[1], np.concatenate(out))
"""


def test_split_sig12_matches_the_monolithic_kernel(tmp_path):
    """The 12-lane pairing in three kernels (k_sig12_miller, the batched norm
    inversion k_sig12_ninv, k_sig12_fe: the default for unpadded launches) and
    in one (k_verify_sig12: padded launches, and every launch with
    HG_SIG12_SPLIT=0) write byte-identical FE values, both kernels 2 and 3 in
    both settings, both flavors, ragged n (a 1029-check batch spans five
    inversion blocks, the last one partly empty), with a point at infinity in
    the batch. Each form runs in a child process (the switch is read once per
    process)."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    got = {}
    for split in ("1", "0"):
        path = str(tmp_path / f"fe_{split}.npy")
        env = dict(os.environ, HG_SIG12_SPLIT=split, HG_ROOT=root)
        r = subprocess.run([sys.executable, "-c", _MONO_CHILD, path], capture_output=True, text=True, timeout=240,
                           env=env)
        assert r.returncode == 0, r.stderr[-3000:]
        got[split] = np.load(path)
    assert got["1"].size == 2 * 2 * (7 + 1029) * 480
    assert np.array_equal(got["1"], got["0"])
