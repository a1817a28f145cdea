"""Registry files and packet-level batches.

CPU: the simulator's CSV node files (simul/lib/parser.go:105-155) round-trip
through handel_amd.registry, with the reference's field-count and id errors.
GPU: the golden 50-node registry loads from its CSV into the engine, the
golden multisig packets go through BatchVerifier.verify_packets (GPU parse,
then verification) with the golden verdicts, and generated records (GenerateNodes with batched keygen)
carry the oracle's public keys."""

import json
import os

import pytest

from handel_amd import registry as REG

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")


def test_csv_roundtrip(tmp_path):
    recs = REG.read_records(os.path.join(GOLD, "registry_50.csv"))
    assert len(recs) == 50 and [r.id for r in recs] == list(range(50))
    out = tmp_path / "reg.csv"
    REG.write_records(str(out), recs)
    with open(os.path.join(GOLD, "registry_50.csv")) as a, open(out) as b:
        assert a.read() == b.read()
    assert len(REG.registry_bytes(recs)) == 50 * 128


def test_csv_errors():
    with pytest.raises(REG.RegistryError, match="wrong number of fields"):
        REG.read_records("0,127.0.0.1:3000,ab\n", is_text=True)
    with pytest.raises(REG.RegistryError, match="invalid syntax"):
        REG.read_records("x,127.0.0.1:3000,ab,cd\n", is_text=True)
    with pytest.raises(REG.RegistryError, match="out of range"):
        REG.read_records("4294967296,a,b,c\n", is_text=True)
    recs = REG.read_records("1,a,01,00\n", is_text=True)
    with pytest.raises(REG.RegistryError, match="ids 0..N-1"):
        REG.registry_bytes(recs)


def test_secret_marshal_is_minimal():
    assert REG.secret_marshal(1) == b"\x01"
    assert REG.secret_marshal(256) == b"\x01\x00"
    assert REG.secret_marshal(REG.ORDER - 1).hex() == hex(REG.ORDER - 1)[2:]


@pytest.mark.gpu
def test_golden_registry_and_packets(engine):
    from handel_amd.processing import BatchVerifier

    with open(os.path.join(GOLD, "bn256_vectors.json")) as f:
        gv = json.load(f)
    ms = gv["multisig"]
    recs = REG.read_records(os.path.join(GOLD, "registry_50.csv"))
    assert REG.load_registry(engine, recs) == 50
    bv = BatchVerifier(engine, REG.registry_bytes(recs), bytes.fromhex(ms["msg"]), node_id=ms["node"])
    reqs = [r for r in ms["requests"] if r["level"] is not None]  # level None: VerifyMultiSignature
    packets = [(r["level"], bytes.fromhex(r["multisig"])) for r in reqs]
    packets.append((1, b"\x00"))                                   # truncated length prefix
    packets.append((1, bytes.fromhex(ms["requests"][0]["multisig"])[:-1]))  # short signature
    got = bv.verify_packets(packets)
    # a packet carries its request through Handel.NewPacket first: a bitset of
    # the wrong size or with no bit set is dropped at parse with its own text
    # (handel.go:398-405) before processing's checks could see it
    want_text = {0: None, 1: "handel: bn256: signature invalid", 3: "invalid bitset's size for given level",
                 6: "no signature in the bitset"}
    for r, g in zip(reqs, got):
        assert g == want_text[r["code"]], (r["level"], r["code"], g)
    assert got[-2] == "unexpected EOF"  # binary.Read of the u16 length from one byte
    assert got[-1] == "bn256: multisig can't unmarshal"


@pytest.mark.gpu
def test_generate_records_match_oracle(engine):
    from oracle import bn256_oracle as O

    r = O.SeededReader(b"registry-gen")
    recs = REG.generate_records(engine, [f"127.0.0.1:{3000 + i}" for i in range(6)], r.read_full)
    r2 = O.SeededReader(b"registry-gen")
    for rec in recs:
        k, err = O.random_scalar(r2)
        assert err is None
        assert rec.private == REG.secret_marshal(k).hex()
        assert rec.public == O.g2_marshal(O.g2_mul(O.G2_GEN, k)).hex()


@pytest.mark.gpu
def test_verify_multisignature_errors(engine):
    """VerifyMultiSignature (crypto.go:120-137) through hg_verify_multisig: the
    full-registry request of the golden set verifies, a bitset of the wrong
    length gets the reference's "inconsistent sizes" text, a tampered
    signature the unwrapped VerifySignature error."""
    from handel_amd import partitioner as part
    from handel_amd.processing import BatchVerifier

    with open(os.path.join(GOLD, "bn256_vectors.json")) as f:
        ms = json.load(f)["multisig"]
    recs = REG.read_records(os.path.join(GOLD, "registry_50.csv"))
    bv = BatchVerifier(engine, REG.registry_bytes(recs), bytes.fromhex(ms["msg"]), node_id=ms["node"])
    full = [r for r in ms["requests"] if r["level"] is None][0]
    bits, sig = part.multisig_unmarshal(bytes.fromhex(full["multisig"]))
    bits = [bool(b) for b in bits]
    assert len(bits) == 50 and sig == bytes.fromhex(full["agg_sig"])
    bad = bytearray(sig)
    bad[5] ^= 1
    got = bv.verify_multisignatures([(bits, sig), (bits[:-1], sig), (bits + [True], sig), (bits, bytes(bad))])
    assert got[0] is None
    assert got[1] == got[2] == "verify multisignature: inconsistent sizes"
    assert got[3] in ("bn256: multisig can't unmarshal", "bn256: signature invalid")
