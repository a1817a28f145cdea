"""CPU suite: the verifier service's shared-memory protocol (hg_service_*,
include/handel_client.h) served by the CPU echo stand-in — no GPU.

What is checked here is the transport between client processes and the one
GPU-owning process (simul/node/main.go:63-131: P processes of k Handel
instances; processing.go:228-287: one check per instance at a time): every
request's bytes arrive intact (the echo code is a checksum of the bitset
words the server received), every code returns to the handle that submitted
it, nothing is lost or duplicated under many concurrent processes, and the
edge cases fail loudly. Verdict parity is the GPU suite's job
(tests/test_gpu_service.py).
"""

import json
import os
import subprocess
import threading

import numpy as np
import pytest

from handel_amd import _lib
from handel_amd import build as B
from handel_amd.service import Client, EchoService, echo_signature, service_name
from tests.test_abi import declared_symbols

MSG = b"handel service test"


def test_client_library_exports_its_header_and_needs_no_gpu_runtime():
    import ctypes

    path = B.build_client(verbose=False)
    lib = ctypes.CDLL(path)
    for s in declared_symbols("handel_client.h"):
        assert hasattr(lib, s), s
    needed = subprocess.run(["readelf", "-d", path], capture_output=True, text=True, check=True).stdout
    assert "amdhip" not in needed and "hsa" not in needed, needed
    from handel_amd.service import CLIENT_SIGNATURES
    assert set(CLIENT_SIGNATURES) == declared_symbols("handel_client.h")


def _req(rng, nreg, words_out):
    """a random request of the echo rule: level range, bitset, signature"""
    size = int(rng.choice([s for s in (1, 2, 7, 64, 65, 128, 500, nreg) if s <= nreg]))
    off = int(rng.integers(0, nreg - size + 1))
    nw = (size + 63) // 64
    w = rng.integers(0, 2**63, size=nw, dtype=np.uint64)
    tampered = bool(rng.integers(0, 2))
    words_out.append(w)
    return off, size, w, echo_signature(w, tampered), (1 if tampered else 0)


def test_echo_service_round_trip_in_process():
    name = service_name("echo1")
    with EchoService(name, nreg=600, delay_us=100, lanes=4, max_wait_us=20) as svc, Client(name) as cl:
        assert cl.slot_bits >= 600
        rng = np.random.default_rng(1)
        ws = []
        want, tickets = [], []
        for _ in range(300):
            off, size, w, sig, exp = _req(rng, 600, ws)
            tickets.append(cl.submit(MSG, off, size, size, w, sig))
            want.append(exp)
        got = [cl.wait(t) for t in reversed(tickets)][::-1]
        assert got == want
        # the level check and a corrupted word
        w = np.arange(2, dtype=np.uint64)
        assert cl.verify(MSG, 590, 100, 100, w, echo_signature(w)) == _lib.HG_ERR_LEVEL
        assert cl.verify(MSG, 0, 100, 99, w, echo_signature(w)) == _lib.HG_ERR_LEVEL
        assert cl.verify(MSG, 0, 100, 100, w, echo_signature(w + 1)) == 77
        b, r, f = svc.stats()
        assert r == 303 and 1 <= b <= 303 and 1 <= f <= 4
        assert cl.stats() == (b, r)


def test_wait_any_collects_every_ticket_once():
    name = service_name("echo2")
    with EchoService(name, nreg=256, delay_us=50, lanes=2), Client(name) as cl:
        rng = np.random.default_rng(2)
        want = {}
        for _ in range(500):
            off, size, w, sig, exp = _req(rng, 256, [])
            want[cl.submit(MSG, off, size, size, w, sig)] = exp
        got = {}
        while len(got) < len(want):
            for t, c in cl.wait_any(cap=64, timeout_us=2_000_000):
                assert t not in got
                got[t] = c
        assert got == want
        assert cl.wait_any(cap=8, timeout_us=1000) == []  # nothing left: timeout


def test_many_threads_share_one_handle():
    name = service_name("echo3")
    errors = []
    with EchoService(name, nreg=1024, delay_us=30, lanes=4), Client(name) as cl:
        def worker(seed):
            rng = np.random.default_rng(seed)
            for _ in range(60):
                off, size, w, sig, exp = _req(rng, 1024, [])
                c = cl.verify(MSG, off, size, size, w, sig)
                if c != exp:
                    errors.append((seed, c, exp))

        th = [threading.Thread(target=worker, args=(s,)) for s in range(8)]
        for t in th:
            t.start()
        for t in th:
            t.join()
    assert not errors


def test_messages_are_batched_apart():
    """Requests under different messages never share a batch; each keeps its code."""
    name = service_name("echo4")
    with EchoService(name, nreg=128, delay_us=20, lanes=2, max_wait_us=200) as svc, Client(name) as cl:
        rng = np.random.default_rng(3)
        want, tickets = [], []
        for i in range(90):
            off, size, w, sig, exp = _req(rng, 128, [])
            tickets.append(cl.submit(b"msg %d" % (i % 3), off, size, size, w, sig))
            want.append(exp)
        assert [cl.wait(t) for t in tickets] == want
        assert svc.stats()[0] >= 3


def test_edge_cases_fail_loudly():
    from handel_amd._lib import HandelGPUError

    with pytest.raises(HandelGPUError):
        Client("/hg_no_such_service_%d" % os.getpid())
    name = service_name("echo5")
    svc = EchoService(name, nreg=100, delay_us=10, slot_bits=128)
    with pytest.raises(HandelGPUError):
        EchoService(name, nreg=100)  # the name is taken
    cl = Client(name)
    w = np.zeros(3, dtype=np.uint64)
    with pytest.raises(HandelGPUError):  # longer than the region's slots
        cl.submit(MSG, 0, 129, 129, w, echo_signature(w))
    with pytest.raises(HandelGPUError):  # message too long
        cl.submit(b"x" * 1025, 0, 1, 1, w[:1], echo_signature(w[:1]))
    with pytest.raises(ValueError):  # fewer words than bits
        cl.submit(MSG, 0, 65, 65, w[:1], echo_signature(w[:1]))
    with pytest.raises(HandelGPUError):
        cl.wait(12345)  # never issued
    with pytest.raises(HandelGPUError):
        cl.wait((999 << 32) | 5)  # a slot of the region, not a ticket of this handle
    # an empty bitset request travels (bitlen 0: no words)
    assert cl.verify(MSG, 0, 0, 0, np.zeros(0, dtype=np.uint64), echo_signature([])) == 0
    # queued requests are verified by the stop; later submissions are refused
    t = cl.submit(MSG, 0, 64, 64, w[:1], echo_signature(w[:1], True))
    svc.close()
    assert cl.wait(t) == _lib.HG_ERR_SIG_INVALID
    with pytest.raises(HandelGPUError):
        cl.submit(MSG, 0, 64, 64, w[:1], echo_signature(w[:1]))
    with pytest.raises(HandelGPUError):
        cl.wait_any(cap=4, timeout_us=1000)  # stopped, nothing left
    cl.close()


def test_channels_are_reused_after_close():
    name = service_name("echo6")
    with EchoService(name, nreg=64, channels=2):
        a, b = Client(name), Client(name)
        from handel_amd._lib import HandelGPUError
        with pytest.raises(HandelGPUError):
            Client(name)  # both channels taken
        a.close()
        c = Client(name)
        w = np.ones(1, dtype=np.uint64)
        assert c.verify(MSG, 0, 64, 64, w, echo_signature(w)) == 0
        c.close()
        b.close()


@pytest.mark.parametrize("procs,pollers", [(4, 1), (3, 2)])
def test_proxy_many_processes_over_the_echo_service(procs, pollers):
    """The config-4 process model over the service: `procs` client processes
    (no GPU library loaded), each with `pollers` handles driving 40 instances
    that check one request at a time; every code comes back to the right
    instance (the proxy compares each with the expected verdict)."""
    exe = B.build_proxy(verbose=False)
    B.build_client(verbose=False)
    r = subprocess.run([exe, B.LIB, "-E", "200", "-p", str(procs), "-k", "40", "-n", "300", "-r", "6", "-w",
                        str(pollers), "-l", "4"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-2000:])
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["model"] == "daemon-echo" and out["mismatches"] == 0
    assert out["requests"] == procs * 40 * 6
    assert out["batches"] < out["requests"]


def _start_verifierd(args):
    exe = B.build_verifierd(verbose=False)
    p = subprocess.Popen([exe, *args], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    line = p.stdout.readline()
    assert line, p.stderr.read()
    return p, json.loads(line)


def test_verifierd_echo_serves_until_sigterm():
    """hg_verifierd: the daemon a single-host run starts once; SIGTERM verifies
    what is queued, prints its statistics and exits 0."""
    import signal

    name = service_name("vd")
    p, ready = _start_verifierd(["--name", name, "--echo", "50", "--nreg", "400", "--lanes", "2"])
    try:
        assert ready["ready"] == name and ready["registry"] == 400
        with Client(name) as cl:
            rng = np.random.default_rng(5)
            want, tickets = [], []
            for _ in range(64):
                off, size, w, sig, exp = _req(rng, 400, [])
                tickets.append(cl.submit(MSG, off, size, size, w, sig))
                want.append(exp)
            assert [cl.wait(t) for t in tickets] == want
            assert cl.processing_error_string(1) == "handel: bn256: signature invalid"
            assert cl.code_string(3) == "handel: inconsistent bitset with given level"
    finally:
        p.send_signal(signal.SIGTERM)
        out, err = p.communicate(timeout=30)
    assert p.returncode == 0, err
    stats = json.loads(out.strip().splitlines()[-1])
    assert stats["stopped"] == name and stats["requests"] == 64


def test_verifierd_rejects_bad_arguments(tmp_path):
    exe = B.build_verifierd(verbose=False)
    assert subprocess.run([exe], capture_output=True).returncode == 2
    bad = tmp_path / "reg.bin"
    bad.write_bytes(bytes(100))  # not a multiple of 128
    r = subprocess.run([exe, "--name", service_name("vd2"), "--registry", str(bad)], capture_output=True, text=True)
    assert r.returncode == 2 and "128-byte" in r.stderr
