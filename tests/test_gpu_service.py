"""GPU suite: the verifier service (hg_service_*, hg_lane_*; clients through
libhandel_client.so) — one GPU-owning context serving the checks of other
threads and processes (simul/node/main.go:63-131, processing.go:228-287).

Every verdict that comes back through the shared-memory region must be the C
restatement's (oracle/bn256_ref.c) for the same request, at table level 2
(prepared) and on the volume policy's G2 fold, with several batches in
flight on separate lanes, with messages interleaved (the context's two-message
table cache), and for a message hashedMessage rejects.
"""

import json
import subprocess

import numpy as np
import pytest

from handel_amd import _lib
from handel_amd import build as B
from handel_amd.engine import REQ_DTYPE, Engine
from handel_amd.service import Client, Service, service_name
from oracle import ref_lib as R
from tests import _fixtures as F
from tests.test_gpu_gt import _batch, _levels, _oracle

pytestmark = pytest.mark.gpu
NREG = 300


@pytest.fixture(scope="module")
def reg300():
    ks, pks, _ = F.keys_and_sigs(NREG, seed=b"service")
    return ks, pks


def _engine(pks, level=-1):
    e = Engine(device=0, flavor="go")
    e.set_aggregate_level(level)
    e.registry_load(pks)
    return e


@pytest.mark.parametrize("prepare", [1, 0], ids=["prepared", "policy"])
def test_service_verdicts_match_oracle(reg300, prepare):
    ks, pks = reg300
    rng = np.random.default_rng(40 + prepare)
    ranges = _levels(NREG, rng.integers(0, NREG, size=12)) * 6
    reqs, words, sigs = _batch(ks, NREG, F.LIB_MESSAGE, ranges, rng)
    want = _oracle(F.LIB_MESSAGE, pks, reqs, words, sigs)
    e = _engine(pks)
    name = service_name("gpu1")
    try:
        with Service(e, name, lanes=4, max_wait_us=30, prepare=prepare) as svc, Client(name) as cl:
            got = cl.verify_many(F.LIB_MESSAGE, reqs, words, sigs)
            assert np.array_equal(got, want)
            assert (got == _lib.HG_ERR_SIG_INVALID).any() and (got == 0).any()
            b, r, f = svc.stats()
            assert r == len(reqs) and b >= 1 and f >= 1
        assert e.aggregate_tables() == (2 if prepare else 0)
    finally:
        e.close()


def test_service_interleaved_messages_and_hash_reject(reg300):
    ks, pks = reg300
    rng = np.random.default_rng(7)
    m1, m2 = F.LIB_MESSAGE, F.TEST_MESSAGES[0]
    ranges = _levels(NREG, rng.integers(0, NREG, size=6)) * 3
    r1, w1, s1 = _batch(ks, NREG, m1, ranges, rng)
    r2, w2, s2 = _batch(ks, NREG, m2, ranges, rng)
    want1, want2 = _oracle(m1, pks, r1, w1, s1), _oracle(m2, pks, r2, w2, s2)
    e = _engine(pks)
    name = service_name("gpu2")
    try:
        with Service(e, name, lanes=3, max_wait_us=200, prepare=1), Client(name) as cl:
            t1, t2 = [], []
            for i in range(len(r1)):  # alternate the two messages request by request
                for reqs, words, sigs, msg, ts in ((r1, w1, s1, m1, t1), (r2, w2, s2, m2, t2)):
                    q = reqs[i]
                    nw = (int(q["bitlen"]) + 63) // 64
                    wo = int(q["word_offset"])
                    ts.append(cl.submit(msg, int(q["offset"]), int(q["bitlen"]), int(q["level_size"]),
                                        words[wo:wo + nw], sigs[64 * i:64 * i + 64]))
            got1 = np.array([cl.wait(t) for t in t1])
            got2 = np.array([cl.wait(t) for t in t2])
            assert np.array_equal(got1, want1) and np.array_equal(got2, want2)
            # both messages kept their tables: level 2 after the switches
            assert e.aggregate_tables() == 2
            # a message hashedMessage rejects: every verdict is its EOF
            bad = F.REJECT_MESSAGES[0]
            codes = cl.verify_many(bad, r1[:5], w1, s1[:5 * 64])
            assert (codes == _lib.HG_ERR_HASH_EOF).all()
    finally:
        e.close()


@pytest.mark.parametrize("level,lanes", [(2, 8), (0, 4)])
def test_proxy_daemon_verdicts_match_oracle(tmp_path, level, lanes):
    """handel_proxy -D 1: one server process (the GPU context), 3 client
    processes that never load the HIP library, 24 instances each checking one
    multisignature at a time; process 0's verdicts against the oracle."""
    exe = B.build_proxy(verbose=False)
    B.build_client(verbose=False)
    cmd = [exe, B.LIB, "-D", "1", "-p", "3", "-k", "24", "-n", "300", "-r", "5", "-L", str(level), "-P", "1",
           "-l", str(lanes), "-d", str(tmp_path)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-2000:])
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["model"] == "daemon" and out["contexts"] == 1
    assert out["mismatches"] == 0 and out["requests"] == 3 * 24 * 5
    assert out["tables_after"] == level
    reg = (tmp_path / "reg.bin").read_bytes()
    reqs = np.frombuffer((tmp_path / "reqs.bin").read_bytes(), dtype=REQ_DTYPE)
    words = np.frombuffer((tmp_path / "words.bin").read_bytes(), dtype=np.uint64)
    sigs = (tmp_path / "sigs.bin").read_bytes()
    got = np.frombuffer((tmp_path / "codes.bin").read_bytes(), dtype=np.int32)
    want = R.verify_aggregate(F.LIB_MESSAGE, reg, reqs["offset"], reqs["bitlen"], reqs["level_size"], words,
                              reqs["word_offset"].astype(np.uint64), sigs, nthreads=8)
    assert np.array_equal(got, want)
    assert (got == 1).sum() == (len(got) + 7) // 8


def test_verifierd_serves_registry_file(tmp_path, reg300):
    """hg_verifierd with --registry/--message (the daemon a simul host starts):
    tables built before "ready", verdicts through a client equal the oracle's,
    SIGTERM prints the statistics and exits 0."""
    import signal

    ks, pks = reg300
    (tmp_path / "reg.bin").write_bytes(pks)
    (tmp_path / "msg.bin").write_bytes(F.LIB_MESSAGE)
    rng = np.random.default_rng(11)
    reqs, words, sigs = _batch(ks, NREG, F.LIB_MESSAGE, _levels(NREG, rng.integers(0, NREG, size=8)) * 4, rng)
    want = _oracle(F.LIB_MESSAGE, pks, reqs, words, sigs)
    name = service_name("vdgpu")
    exe = B.build_verifierd(verbose=False)
    p = subprocess.Popen([exe, "--name", name, "--registry", str(tmp_path / "reg.bin"), "--message",
                          str(tmp_path / "msg.bin"), "--lanes", "3"], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                         text=True)
    try:
        ready = json.loads(p.stdout.readline() or "{}")
        assert ready.get("ready") == name and ready["registry"] == NREG and ready["tables"] == 2, p.stderr.read()
        with Client(name) as cl:
            assert cl.flavor == 0
            got = cl.verify_many(F.LIB_MESSAGE, reqs, words, sigs)
        assert np.array_equal(got, want)
    finally:
        p.send_signal(signal.SIGTERM)
        out, err = p.communicate(timeout=60)
    assert p.returncode == 0, err
    stats = json.loads(out.strip().splitlines()[-1])
    assert stats["requests"] == len(reqs) and stats["tables"] == 2
