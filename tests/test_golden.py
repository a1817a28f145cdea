"""Golden vectors (tests/golden/, made by tests/golden/make_golden.py).

CPU: the committed vectors are reproduced by the Python oracle (the generator
is re-run into a temp dir), the C restatement matches every vector, and the
host-side mirrors (partitioner, bitset/multisig wire format, registry CSV
parser) agree with them. GPU: every engine entry point reproduces the vectors
byte for byte through the C ABI.
"""

import csv
import importlib.util
import json
import os

import numpy as np
import pytest

from oracle import bn256_oracle as O
from oracle import ref_lib as R

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")


@pytest.fixture(scope="module")
def gv():
    with open(os.path.join(GOLD, "bn256_vectors.json")) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def registry():
    with open(os.path.join(GOLD, "registry_50.csv")) as f:
        rows = list(csv.reader(f))
    return [(int(r[0]), r[1], bytes.fromhex(r[2]), bytes.fromhex(r[3])) for r in rows]


def b(h):
    return bytes.fromhex(h)


# ------------------------------------------------------------------ CPU
def test_generator_reproduces_committed_vectors(tmp_path, monkeypatch):
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(GOLD, "make_golden.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    monkeypatch.setattr(mod, "HERE", str(tmp_path))
    mod.main()
    for name in ("bn256_vectors.json", "registry_50.csv"):
        with open(os.path.join(GOLD, name), "rb") as f1, open(tmp_path / name, "rb") as f2:
            assert f1.read() == f2.read(), name


def test_c_restatement_matches_golden(gv):
    # pairing GT bytes
    for v in gv["pair"]:
        assert R.pair(b(v["g1"]), b(v["g2"])) == b(v["gt"])
    # keygen / sign
    s = gv["sign"]
    kb = b"".join(b(k).rjust(32, b"\0") for k in s["sk"])
    assert R.g2_scalar_base(kb) == b"".join(b(p) for p in s["pk"])
    assert R.sign(b(s["msg"]), kb) == b"".join(b(x) for x in s["sig"])
    # verification codes (grouped by message)
    by_msg = {}
    for v in gv["verify"]:
        by_msg.setdefault(v["msg"], []).append(v)
    for m, vs in by_msg.items():
        codes = R.verify_batch(b(m), b"".join(b(v["pk"]) for v in vs), b"".join(b(v["sig"]) for v in vs),
                               nthreads=4)
        assert list(codes) == [v["code"] for v in vs]
        fast = R.verify_batch(b(m), b"".join(b(v["pk"]) for v in vs), b"".join(b(v["sig"]) for v in vs),
                              nthreads=4, fast=2)
        assert list(fast) == [v["code"] for v in vs]
    for v in gv["combine_g1"]:
        assert R.g1_add(b(v["a"]), b(v["b"])) == b(v["out"])
    for v in gv["combine_g2"]:
        assert R.g2_add(b(v["a"]), b(v["b"])) == b(v["out"])


def test_c_restatement_aggregate_matches_golden(gv, registry):
    ms = gv["multisig"]
    reg = b"".join(r[3] for r in registry)
    reqs = ms["requests"]
    words, woff = [], []
    for q in reqs:
        bits = O.bitset_unmarshal(b(q["bitset"]))
        woff.append(len(words))
        words.extend(O.bitset_words(bits))
    codes, agg = R.verify_aggregate(b(ms["msg"]), reg, [q["lo"] for q in reqs], [q["bitlen"] for q in reqs],
                                    [q["hi"] - q["lo"] for q in reqs], np.array(words, dtype=np.uint64),
                                    np.array(woff, dtype=np.uint64), b"".join(b(q["agg_sig"]) for q in reqs),
                                    nthreads=4, want_agg=True)
    assert list(codes) == [q["code"] for q in reqs]
    for i, q in enumerate(reqs):
        if q["agg_pk"] is not None:
            assert agg[128 * i:128 * i + 128] == b(q["agg_pk"])


def test_python_oracle_matches_golden_unmarshal(gv):
    for u in gv["unmarshal"]:
        fn = O.g1_unmarshal if u["kind"] == "g1" else O.g2_unmarshal
        _, err = fn(b(u["bytes"]), u["flavor"])
        assert err == u["err"]


def test_host_mirrors_match_golden(gv, registry):
    from handel_amd import partitioner as part

    for v in gv["range_level_4000"]:
        try:
            got = list(part.range_level(v["id"], 4000, v["level"]))
        except part.PartitionerError as e:
            got = None
            assert v["err"] is not None, str(e)
        assert got == v["range"]
    for q in gv["multisig"]["requests"]:
        bits, sig = part.multisig_unmarshal(b(q["multisig"]))
        assert len(bits) == q["bitlen"] and sig == b(q["agg_sig"])
        assert part.multisig_marshal(bits, sig) == b(q["multisig"])
        assert part.bitset_marshal(bits) == b(q["bitset"])
    # registry CSV: ids dense, sk marshal minimal big-endian, pk = sk * G2 (the golden 'sign' table)
    s = gv["sign"]
    assert [r[0] for r in registry] == list(range(50))
    assert [r[2].hex() for r in registry] == s["sk"]
    assert [r[3].hex() for r in registry] == s["pk"]


# ------------------------------------------------------------------ GPU (through the C ABI)
@pytest.mark.gpu
def test_gpu_pair_keygen_sign_golden(engine, gv):
    for v in gv["pair"]:
        gt, codes = engine.pair(b(v["g1"]), b(v["g2"]))
        assert gt == b(v["gt"]) and list(codes) == [0]
    s = gv["sign"]
    kb = b"".join(b(k).rjust(32, b"\0") for k in s["sk"])
    assert engine.set_message(b(s["msg"])) == 0
    assert engine.keygen(kb) == b"".join(b(p) for p in s["pk"])
    assert engine.sign(kb) == b"".join(b(x) for x in s["sig"])


@pytest.mark.gpu
def test_gpu_verify_golden(engine, gv):
    by_msg = {}
    for v in gv["verify"]:
        by_msg.setdefault(v["msg"], []).append(v)
    for m, vs in by_msg.items():
        engine.set_message(b(m))
        got = engine.verify_batch(b"".join(b(v["pk"]) for v in vs), b"".join(b(v["sig"]) for v in vs))
        assert list(got) == [v["code"] for v in vs]


@pytest.mark.gpu
def test_gpu_hash_and_combine_golden(engine, gv):
    for h in gv["hash"]:
        assert engine.set_message(b(h["msg"])) == h["code"]
    for v in gv["combine_g1"]:
        out, codes = engine.combine_g1(b(v["a"]), b(v["b"]))
        assert out == b(v["out"]) and list(codes) == [0]
    for v in gv["combine_g2"]:
        out, codes = engine.combine_g2(b(v["a"]), b(v["b"]))
        assert out == b(v["out"]) and list(codes) == [0]


@pytest.mark.gpu
def test_gpu_multisig_golden(engine, gv, registry):
    from handel_amd.processing import BatchVerifier

    ms = gv["multisig"]
    bv = BatchVerifier(engine, b"".join(r[3] for r in registry), b(ms["msg"]), node_id=ms["node"])
    items = []
    for q in ms["requests"]:
        bits = O.bitset_unmarshal(b(q["bitset"]))
        items.append((q["lo"], q["hi"] - q["lo"], bits, b(q["agg_sig"])))
    (reqs, words, sigs), pre, _ = bv._pack(items)
    assert not pre.any()  # every golden signature is 64 bytes
    codes, agg = engine.verify_aggregate(reqs, words, sigs, want_agg=True)
    assert list(codes) == [q["code"] for q in ms["requests"]]
    for i, q in enumerate(ms["requests"]):
        if q["agg_pk"] is not None and q["code"] in (0, 1):
            assert agg[128 * i:128 * i + 128] == b(q["agg_pk"])


@pytest.mark.gpu
def test_gpu_g2_unmarshal_golden(engine, engine_cf, gv):
    """Registry decode applies each flavor's PublicKey.UnmarshalBinary rule
    (bn256/go/bn256.go:113-120, bn256/cf/bn256.go:112-121)."""
    cf_codes = {O.ERR_CF_EXCEEDS: 7, O.ERR_CF_MALFORMED: 8, O.ERR_CF_NOT_ENOUGH: 9}
    for flavor, eng in (("go", engine), ("cf", engine_cf)):
        cases = [u for u in gv["unmarshal"] if u["kind"] == "g2" and u["flavor"] == flavor
                 and len(u["bytes"]) == 256]
        got = eng.registry_load(b"".join(b(u["bytes"]) for u in cases))
        want = [0 if u["err"] is None else (4 if flavor == "go" else cf_codes[u["err"]]) for u in cases]
        assert list(got) == want, flavor
