"""Packet intake on the GPU (hg_parse_packets / hg_parse_packets_device)
against the restatement of Handel.NewPacket's parse step
(oracle.bn256_oracle.parse_packet: handel.go:371-436, crypto.go:86-110,
bitset.go:166-177, willf/bitset v1.1.10 ReadFrom): the committed vectors, a
4096-packet batch of well-formed and damaged packets per flavor, and packets
parsed in HBM feeding hg_verify_aggregate_device end to end."""

import json
import os
import random

import numpy as np
import pytest

from oracle import bn256_oracle as O

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _engine(nreg: int, flavor: str):
    import bench
    from handel_amd.engine import Engine

    e = Engine(device=0, flavor=flavor)
    assert not e.registry_load(e.keygen(bench.seeded_scalars(nreg, 77 + nreg))).any()
    return e


def _check_batch(eng, cases):
    """cases: dicts with nreg/flavor/receiver/origin/level/ms/ind (bytes) and
    the oracle's result under "want"; parses them in one call and compares
    every output slot."""
    from handel_amd import _lib
    from handel_amd.packets import Packet, pack_packets

    pkts = [Packet(c["origin"], c["level"], c["ms"], c["ind"]) for c in cases]
    pool, recs = pack_packets(pkts, [c["receiver"] for c in cases])
    reqs, words, sigs, codes = eng.parse_packets(pool, recs)
    n = len(cases)
    for i, c in enumerate(cases):
        w = c["want"]
        code = int(codes[i])
        got_err = "" if code == _lib.HG_OK else eng.packet_error(code, recs[i])
        assert got_err == (w["err"] or ""), (i, c.get("name"), got_err, w["err"])
        if code != _lib.HG_OK:
            assert int(codes[n + i]) == code
            continue
        r = reqs[i]
        lo, hi = w["range"]
        assert (int(r["offset"]), int(r["bitlen"]), int(r["level_size"])) == (lo, w["bitlen"], hi - lo), i
        nw = (w["bitlen"] + 63) // 64
        wo = int(r["word_offset"])
        v = sum(int(x) << (64 * j) for j, x in enumerate(words[wo:wo + nw]))
        assert v == w["bits"], (i, c.get("name"))
        assert sigs[64 * i:64 * i + 64] == w["sig"][:64]
        ri = reqs[n + i]
        if w["ind_bit"] is None:
            assert int(codes[n + i]) == _lib.HG_PKT_NO_IND
        else:
            assert int(codes[n + i]) == _lib.HG_OK
            assert (int(ri["offset"]), int(ri["bitlen"]), int(ri["level_size"])) == (lo, hi - lo, hi - lo)
            wo2 = int(ri["word_offset"])
            v2 = sum(int(x) << (64 * j) for j, x in enumerate(words[wo2:wo2 + (hi - lo + 63) // 64]))
            assert v2 == 1 << w["ind_bit"]
            assert sigs[64 * (n + i):64 * (n + i) + 64] == c["ind"][:64]


def test_golden_packets():
    with open(os.path.join(HERE, "golden", "packet_vectors.json")) as f:
        cases = json.load(f)["cases"]
    groups = {}
    for c in cases:
        groups.setdefault((c["nreg"], c["flavor"]), []).append(
            {"name": c["name"], "receiver": c["receiver"], "origin": c["origin"], "level": c["level"],
             "ms": bytes.fromhex(c["ms"]), "ind": None if c["ind"] is None else bytes.fromhex(c["ind"]),
             "want": {"err": c["err"], "range": tuple(c["range"]), "bitlen": c["bitlen"], "bits": int(c["bits"], 16),
                      "sig": bytes.fromhex(c["sig"]), "ind_bit": c["ind_bit"]}})
    for (nreg, flavor), cs in groups.items():
        e = _engine(nreg, flavor)
        try:
            _check_batch(e, cs)
        finally:
            e.close()


def _damaged_batch(n_pkts: int, nreg: int, flavor: str, seed: int):
    """Handel-shaped packets (random receiver, level, density, origin, optional
    individual signature), a third of them damaged in one place: cut short,
    a length field changed, a signature byte flipped, the bitset emptied, the
    level or origin changed."""
    rnd = random.Random(seed)
    pts = [O.g1_marshal(O.g1_mul(O.G1_GEN, k)) for k in range(2, 14)]
    cases = []
    for t in range(n_pkts):
        recv = rnd.randrange(nreg)
        levels = [l for l in range(1, O.log2_ceil(nreg) + 1) if O.range_level(recv, nreg, l)[0]]
        level = rnd.choice(levels)
        lo, hi = O.range_level(recv, nreg, level)[0]
        bits = [rnd.random() < rnd.uniform(0.3, 1.0) for _ in range(hi - lo)]
        ms = bytearray(O.multisig_marshal(bits, O.g1_mul(O.G1_GEN, rnd.randrange(2, 14))))
        origin = rnd.randrange(lo, hi) if rnd.random() < 0.9 else rnd.randrange(-2, nreg + 2)
        ind = pts[t % len(pts)] if rnd.random() < 0.4 else None
        kind = rnd.randrange(12)
        if kind == 0:
            ms = ms[:rnd.randrange(len(ms))]
        elif kind == 1:
            pos = rnd.randrange(12)
            ms[pos] = rnd.randrange(256)
        elif kind == 2:
            pos = len(ms) - 1 - rnd.randrange(64)
            ms[pos] ^= 1 << rnd.randrange(8)
        elif kind == 3:
            ms = bytearray(O.multisig_marshal([False] * (hi - lo), O.g1_mul(O.G1_GEN, 3)))
        elif kind == 4:
            level = rnd.randrange(0, 16)
        elif kind == 5 and ind is not None:
            ind = ind[:rnd.randrange(70)]
        elif kind == 6:
            ms += bytes(rnd.randrange(1, 4))
        cases.append({"receiver": recv, "origin": origin, "level": level, "ms": bytes(ms), "ind": ind})
    for c in cases:
        c["want"] = O.parse_packet(nreg, flavor, c["receiver"], c["origin"], c["level"], c["ms"], c["ind"])
    return cases


@pytest.mark.parametrize("flavor", ["go", "cf"])
def test_damaged_batch_matches_restatement(flavor):
    cases = _damaged_batch(4096, 4000, flavor, seed=11 if flavor == "go" else 12)
    errs = {c["want"]["err"] for c in cases}
    assert len(errs) >= 8  # the damage reaches many different checks
    e = _engine(4000, flavor)
    try:
        _check_batch(e, cases)
    finally:
        e.close()


def test_bad_arguments():
    from handel_amd._lib import HandelGPUError
    from handel_amd.engine import PACKET_DTYPE

    e = _engine(64, "go")
    try:
        recs = np.zeros(1, dtype=PACKET_DTYPE)
        recs[0]["ms_off"], recs[0]["ms_len"] = 0, 10
        with pytest.raises(HandelGPUError):  # range outside the pool
            e.parse_packets(b"123", recs)
        recs[0]["ms_len"] = 3
        with pytest.raises(HandelGPUError):  # slots too narrow for the largest level (32 ids -> 1 word)
            e.parse_packets(b"123", recs, stride=0)
        reqs, words, sigs, codes = e.parse_packets(b"123", recs)
        assert e.packet_stride_words() == 1 and len(words) == 2
        assert e.packet_error(int(codes[0]), recs[0]) in ("invalid packet's level 0", "packet's origin out of range")
    finally:
        e.close()


def _has_range(node: int, nreg: int, level: int, lo: int, size: int) -> bool:
    from handel_amd import partitioner as HP

    if node >= nreg:
        return False
    try:
        return HP.range_level(node, nreg, level) == (lo, lo + size)
    except HP.PartitionerError:
        return False


def test_device_parse_feeds_verification():
    """Packets in HBM -> hg_parse_packets_device -> hg_verify_aggregate_device
    on the parsed slots: the verdicts are the ones the requests were built
    with (1/8 tampered); no packet carries an individual signature."""
    import torch

    import bench
    from handel_amd import partitioner as HP
    from handel_amd.engine import Engine, PACKET_DTYPE, REQ_DTYPE
    from handel_amd.packets import Packet, pack_packets

    e = Engine(device=0, flavor="go")
    try:
        assert e.set_message(bench.LIB_MESSAGE) == 0
        n_reg, n = 4000, 512
        reqs, words, sigs, expect, _, _ = bench.make_aggregate_batch(e, n_reg, n, seed=91)
        rnd = random.Random(5)
        pkts, recv = [], []
        for i, r in enumerate(reqs):
            lo, size = int(r["offset"]), int(r["level_size"])
            nw = (size + 63) // 64
            bits = HP.words_to_bits(words[int(r["word_offset"]):int(r["word_offset"]) + nw], size)
            # a receiver whose level range is [lo, lo + size): the sibling block
            rv, lv = next((lo ^ (1 << k), k + 1) for k in range(12) if _has_range(lo ^ (1 << k), n_reg, k + 1, lo, size))
            pkts.append(Packet(rnd.randrange(lo, lo + size), lv, HP.multisig_marshal(bits, sigs[64 * i:64 * i + 64])))
            recv.append(rv)
        pool, recs = pack_packets(pkts, recv)
        stride = e.packet_stride_words()
        dev = torch.device("cuda", 0)
        d_pool = torch.from_numpy(np.frombuffer(pool, dtype=np.uint8).copy()).to(dev)
        d_pkts = torch.from_numpy(recs.view(np.uint8).copy()).to(dev)
        d_reqs = torch.zeros(2 * n * REQ_DTYPE.itemsize, dtype=torch.uint8, device=dev)
        d_words = torch.zeros(2 * n * stride, dtype=torch.int64, device=dev)
        d_sigs = torch.zeros(2 * n * 64, dtype=torch.uint8, device=dev)
        d_pcodes = torch.full((2 * n,), -1, dtype=torch.int32, device=dev)
        d_codes = torch.full((n,), -1, dtype=torch.int32, device=dev)
        s = torch.cuda.current_stream(dev).cuda_stream
        e.parse_packets_device(d_pool.data_ptr(), len(pool), d_pkts.data_ptr(), n, stride, d_reqs.data_ptr(),
                               d_words.data_ptr(), d_sigs.data_ptr(), d_pcodes.data_ptr(), s)
        e.verify_aggregate_device(d_reqs.data_ptr(), n, d_words.data_ptr(), d_sigs.data_ptr(), d_codes.data_ptr(),
                                  stream=s)
        torch.cuda.synchronize(dev)
        pc = d_pcodes.cpu().numpy()
        assert (pc[:n] == 0).all() and (pc[n:] == 29).all()  # every packet accepted, none with an individual sig
        assert np.array_equal(d_codes.cpu().numpy(), expect)
        got = np.frombuffer(d_reqs.cpu().numpy().tobytes(), dtype=REQ_DTYPE)[:n]
        assert np.array_equal(got["offset"], reqs["offset"]) and np.array_equal(got["bitlen"], reqs["bitlen"])
        assert PACKET_DTYPE.itemsize == 32
    finally:
        e.close()
