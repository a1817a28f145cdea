"""The drop-in boundary on the GPU: the C ABI's thread-safety and ordering
contract (include/handel_gpu.h), its error paths, the cloudflare flavor's
signature decode, and sharded verification through the engine.

Expected results come from the CPU oracle (oracle/ref_lib, oracle/bn256_oracle)
on the same inputs; integer/byte work, so every comparison is exact.
"""

import os
import socket
import subprocess
import threading

import numpy as np
import pytest

from oracle import bn256_oracle as O
from oracle import ref_lib as R
from tests import _fixtures as F

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MSG2 = F.TEST_MESSAGES[0]


def _req_dtype():
    from handel_amd.engine import REQ_DTYPE
    return REQ_DTYPE


def _aggregate_fixture(n_reg=64, seed=b"abi-threads"):
    """A registry, requests over its Handel level ranges (node 5), aggregate
    signatures on lib.Message (one tampered) and the oracle's results."""
    ks, reg, _ = F.keys_and_sigs(n_reg, seed=seed)
    rng = np.random.default_rng(3)
    ranges = []
    for lvl in range(1, O.log2_ceil(n_reg) + 1):
        rl, err = O.range_level(5, n_reg, lvl)
        if err is None:
            ranges.append((rl[0], rl[1] - rl[0]))
    ranges.append((0, n_reg))
    bitsets = F.random_bitsets(rng, [s for _, s in ranges])
    for b in bitsets:
        b[0] = True
    hm = O.hashed_message(F.LIB_MESSAGE)[0]
    sigs = b""
    for (off, size), bits in zip(ranges, bitsets):
        k = sum(ks[off + i] for i, b in enumerate(bits) if b) % O.ORDER
        sigs += O.g1_marshal(O.g1_mul(hm, k))
    sigs = bytearray(sigs)
    sigs[64:128] = F.tamper(bytes(sigs[64:128]), every=1)
    sigs = bytes(sigs)
    reqs, words = F.pack_requests(ranges, bitsets)
    reqs = np.array(reqs, dtype=_req_dtype())
    codes, agg = R.verify_aggregate(F.LIB_MESSAGE, reg, reqs["offset"], reqs["bitlen"], reqs["level_size"], words,
                                    reqs["word_offset"].astype(np.uint64), sigs, nthreads=4, want_agg=True)
    return reg, reqs, words, sigs, codes, agg


def test_abi_threads_native(engine, tmp_path):
    """tests/native/abi_threads.c: 8 pthreads x 24 calls on ONE context —
    aggregate batches on lib.Message and single-check batches on two different
    messages (hg_*_msg) interleaved — every result equal to the oracle's."""
    from handel_amd import build as B

    exe = B.ABI_THREADS
    assert os.path.exists(exe), "build() compiles the harness in-tree"
    reg, reqs, words, sigs, codes, agg = _aggregate_fixture()
    # the harness's expectations are the oracle's; the GPU agrees single-threaded first
    assert engine.set_message(F.LIB_MESSAGE) == 0
    assert list(engine.registry_load(reg)) == [0] * 64
    got_codes, got_agg = engine.verify_aggregate(reqs, words, sigs, want_agg=True)
    assert list(got_codes) == list(codes) and got_agg == agg
    d = tmp_path
    (d / "reg.bin").write_bytes(reg)
    (d / "reqs.bin").write_bytes(reqs.tobytes())
    (d / "words.bin").write_bytes(words.tobytes())
    (d / "asigs.bin").write_bytes(sigs)
    (d / "acodes.bin").write_bytes(np.asarray(codes, dtype=np.int32).tobytes())
    (d / "agg.bin").write_bytes(agg)
    for k, msg in ((1, F.LIB_MESSAGE), (2, MSG2)):
        _, pks, s = F.keys_and_sigs(24, msg=msg, seed=b"abi-single-%d" % k)
        s = F.tamper(s, every=5)
        want = R.verify_batch(msg, pks, s, nthreads=4)
        (d / f"msg{k}.bin").write_bytes(msg)
        (d / f"pks{k}.bin").write_bytes(pks)
        (d / f"sigs{k}.bin").write_bytes(s)
        (d / f"codes{k}.bin").write_bytes(np.asarray(want, dtype=np.int32).tobytes())
    r = subprocess.run([exe, str(d), "8", "24"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.strip() == "abi_threads ok 192"


def test_verify_signature_threads_different_messages():
    """bn256.PublicKey.VerifySignature from 6 threads on one process-wide
    engine with two messages: hashing and checking are one locked ABI call
    (hg_verify_batch_msg), so no thread sees the other message's H."""
    from handel_amd import bn256 as BN

    ks1, pks1, sigs1 = F.keys_and_sigs(4, msg=F.LIB_MESSAGE, seed=b"thr-1")
    ks2, pks2, sigs2 = F.keys_and_sigs(4, msg=MSG2, seed=b"thr-2")
    cases = []
    for i in range(4):
        cases.append((F.LIB_MESSAGE, pks1[128 * i:128 * i + 128], sigs1[64 * i:64 * i + 64], None))
        cases.append((MSG2, pks2[128 * i:128 * i + 128], sigs2[64 * i:64 * i + 64], None))
        # cross-message pairs must fail
        cases.append((MSG2, pks1[128 * i:128 * i + 128], sigs1[64 * i:64 * i + 64], "bn256: signature invalid"))
    errors = []

    def run(tid):
        for rep in range(6):
            for j, (msg, pk, sig, want) in enumerate(cases):
                if (j + tid + rep) % 2:
                    continue
                e = BN.PublicKey(pk).VerifySignature(msg, BN.SigBLS(sig))
                got = None if e is None else str(e)
                if got != want:
                    errors.append((tid, j, got, want))

    ts = [threading.Thread(target=run, args=(t,)) for t in range(6)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert errors == []


def test_sign_msg_matches_oracle(engine):
    """hg_sign_msg: SecretKey.Sign with the message per call; EOF for a
    message whose digest is >= n (bn256/go/bn256.go:146-154, 210-218)."""
    from handel_amd._lib import HandelGPUError

    ks = F.scalars(5, b"sign-msg")
    kb = F.scalar_bytes(ks)
    assert engine.sign_msg(MSG2, kb) == R.sign(MSG2, kb)
    assert engine.sign_msg(F.LIB_MESSAGE, kb) == R.sign(F.LIB_MESSAGE, kb)
    with pytest.raises(HandelGPUError, match="code 2"):
        engine.sign_msg(F.REJECT_MESSAGES[0], kb)


def test_registry_failure_leaves_no_registry(engine):
    """hg_registry_load with an undecodable key fails AND leaves the context
    without a registry: a later aggregate request cannot read tables of the
    previous registry (it fails the level/range check), and a good reload
    restores service."""
    reg, reqs, words, sigs, codes, _ = _aggregate_fixture()
    assert engine.set_message(F.LIB_MESSAGE) == 0
    assert list(engine.registry_load(reg)) == [0] * 64
    bad = bytearray(reg)
    bad[128 * 7 + 127] ^= 1  # off the curve
    got = engine.registry_load(bytes(bad))
    assert list(np.flatnonzero(got)) == [7] and got[7] == 4
    assert engine.L.hg_registry_size(engine.ctx) == 0
    after = engine.verify_aggregate(reqs, words, sigs)
    assert list(after) == [3] * len(reqs)  # HG_ERR_LEVEL: the range exceeds the (empty) registry
    assert list(engine.registry_load(reg)) == [0] * 64
    assert list(engine.verify_aggregate(reqs, words, sigs)) == list(codes)


def test_submissions_on_two_streams_keep_order(engine):
    """Two asynchronous submissions on ONE context, on two different HIP
    streams, back to back: the second waits for the first (they share the
    context's workspaces), so both batches' verdicts are right."""
    import torch

    import bench

    n = 512
    assert engine.set_message(F.LIB_MESSAGE) == 0
    reqs, words, asigs, aexpect, _, _ = bench.make_aggregate_batch(engine, 300, n, seed=5)
    pks, sigs, sexpect = bench.make_batch(engine, n, seed=6)
    dev = torch.device("cuda", 0)
    t = lambda b: torch.frombuffer(bytearray(b), dtype=torch.uint8).to(dev)  # noqa: E731
    d_reqs, d_words, d_asigs, d_pks, d_sigs = t(reqs.tobytes()), t(words.tobytes()), t(asigs), t(pks), t(sigs)
    a_codes = torch.zeros(n, dtype=torch.int32, device=dev)
    s_codes = torch.zeros(n, dtype=torch.int32, device=dev)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    torch.cuda.synchronize()
    for _ in range(3):
        engine.verify_aggregate_device(d_reqs.data_ptr(), n, d_words.data_ptr(), d_asigs.data_ptr(),
                                       a_codes.data_ptr(), 0, s1.cuda_stream)
        engine.verify_batch_device(d_pks.data_ptr(), d_sigs.data_ptr(), n, s_codes.data_ptr(), s2.cuda_stream)
    torch.cuda.synchronize()
    assert np.array_equal(a_codes.cpu().numpy(), aexpect)
    assert np.array_equal(s_codes.cpu().numpy(), sexpect)


def _cf_sig_cases():
    """(sig bytes, oracle error text or None) for cloudflare's G1 rules."""
    hm = O.hashed_message(MSG2)[0]
    good = O.g1_marshal(O.g1_mul(hm, 12345))
    x = int.from_bytes(good[:32], "big")
    y = int.from_bytes(good[32:], "big")
    cases = [good, bytes(64)]
    cases.append(O.P.to_bytes(32, "big") + good[32:])                    # x == p
    cases.append(good[:32] + (y + O.P).to_bytes(32, "big") if y + O.P < 1 << 256 else good[:32] + b"\xff" * 32)
    cases.append((x ^ 1).to_bytes(32, "big") + good[32:])                # off the curve
    cases.append(b"\xff" * 64)                                           # both >= p
    cases.append((1).to_bytes(32, "big") + (3).to_bytes(32, "big"))      # small, off the curve
    return cases


def test_cf_signature_decode_edge_cases(engine_cf):
    """Cloudflare flavor through hg_verify_batch: coordinates >= p, off-curve
    and infinity signatures get the reference's verdict and error text
    "bn256: multisig can't unmarshal: <cf error>" (bn256/cf/bn256.go:183-190)."""
    ks, pks, _ = F.keys_and_sigs(1, msg=MSG2, seed=b"cf-edge")
    cases = _cf_sig_cases()
    # the valid case signs with the key: replace case 0 by the real signature
    cases[0] = R.sign(MSG2, F.scalar_bytes(ks))
    assert engine_cf.set_message(MSG2) == 0
    got = engine_cf.verify_batch(pks * len(cases), b"".join(cases))
    P_, e1 = O.g2_unmarshal(pks, "cf")
    assert e1 is None
    for i, s in enumerate(cases):
        S, err = O.g1_unmarshal(s, "cf")
        if err is not None:
            want_text = "bn256: multisig can't unmarshal: " + err
            assert engine_cf.code_string(int(got[i])) == want_text, (i, got[i])
        else:
            v = O.verify_signature(P_, MSG2, S)
            assert (got[i] == 0) == (v is None), (i, got[i], v)
    assert got[0] == 0 and got[2] != 0 and got[4] != 0
    assert engine_cf.code_string(int(got[2])) == "bn256: multisig can't unmarshal: bn256: coordinate exceeds modulus"
    assert engine_cf.code_string(int(got[4])) == "bn256: multisig can't unmarshal: bn256: malformed point"


def test_cf_mirror_unmarshal_text():
    """handel_amd.bn256 (cf flavor) SigBLS.UnmarshalBinary raises the wrapped
    cloudflare text; go flavor the bare x/crypto wrapper text."""
    from handel_amd import bn256 as BN

    cf, go = BN.NewConstructor("cf"), BN.NewConstructor("go")
    off = (1).to_bytes(32, "big") + (3).to_bytes(32, "big")  # 9 != 1 + 3
    with pytest.raises(BN.BN256Error, match="^bn256: multisig can't unmarshal: bn256: malformed point$"):
        cf.Signature().UnmarshalBinary(off)
    with pytest.raises(BN.BN256Error, match="^bn256: multisig can't unmarshal$"):
        go.Signature().UnmarshalBinary(off)
    with pytest.raises(BN.BN256Error, match="exceeds modulus"):
        cf.Signature().UnmarshalBinary(b"\xff" * 64)
    # go reduces coordinates mod p; the mirror keeps the reduced re-encoding
    ks, pks, _ = F.keys_and_sigs(1, seed=b"reduce")
    s = go.Signature()
    g1 = O.g1_marshal(O.G1_GEN)
    x = int.from_bytes(g1[:32], "big") + O.P
    s.UnmarshalBinary(x.to_bytes(32, "big") + g1[32:])
    assert s.MarshalBinary() == g1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _sharded_engine_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist

    import bench
    from handel_amd.distributed import verify_sharded
    from handel_amd.engine import Engine

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    eng = Engine(device=0, flavor="go")
    try:
        assert eng.set_message(F.LIB_MESSAGE) == 0
        n = 1000
        # every rank builds the same batch (seeded), then verifies only its slice
        reqs, words, sigs, expect, _, _ = bench.make_aggregate_batch(eng, 200, n, seed=11)

        def verify(lo, hi):
            codes = eng.verify_aggregate(reqs[lo:hi], words, sigs[64 * lo:64 * hi])
            return torch.from_numpy(np.asarray(codes, dtype=np.int32))

        full = verify_sharded(verify, n, rank, world, device=torch.device("cpu"))
        q.put((rank, bool(np.array_equal(full.numpy(), expect == 0)), int(full.sum())))
    finally:
        eng.close()
        dist.destroy_process_group()


def test_sharded_verification_two_ranks_one_gpu():
    """The N>1 path end to end through the engine: 2 ranks (gloo, sharing the
    one GPU of the box) each verify their slice of a config-3 batch on the GPU
    and all-gather verdict bitsets; both end with the whole batch's verdicts."""
    import torch.multiprocessing as mp

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sharded_engine_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
        assert p.exitcode == 0
    res = sorted(q.get(timeout=10) for _ in range(world))
    assert [r[1] for r in res] == [True, True]
    assert res[0][2] == res[1][2] == 1000 - 125


def test_native_batcher_two_messages_threads(engine):
    """hg_batcher_*: 16 threads each verify their own requests one at a time
    (a Handel instance's processLoop) on two interleaved messages; every
    verdict is the one-batch result of hg_verify_aggregate_msg for its
    message, and concurrent requests were merged into fewer launches."""
    import threading

    import bench
    from handel_amd.engine import Batcher

    n_reg, n = 300, 96
    msgs = [bench.LIB_MESSAGE, b"Peaches and Cream"]
    assert engine.set_message(msgs[0]) == 0
    reqs, words, sigs, expect, _, reg = bench.make_aggregate_batch(engine, n_reg, n, seed=31)
    want = [engine.verify_aggregate_msg(m, reqs, words, sigs) for m in msgs]
    assert np.array_equal(want[0], expect) and (want[1] != 0).all()
    b = Batcher(engine, max_batch=64, max_wait_us=500)
    got = [np.full(n, -1, dtype=np.int32) for _ in msgs]
    errors = []

    def instance(t):
        try:
            for i in range(t, n, 16):
                r = reqs[i]
                nw = (int(r["bitlen"]) + 63) // 64
                w = words[int(r["word_offset"]):int(r["word_offset"]) + nw]
                for k in (t % 2, 1 - t % 2):
                    got[k][i] = b.verify(msgs[k], int(r["offset"]), int(r["bitlen"]), int(r["level_size"]), w,
                                         sigs[64 * i:64 * i + 64])
        except Exception as e:  # pragma: no cover - reported below
            errors.append(e)

    ths = [threading.Thread(target=instance, args=(t,)) for t in range(16)]
    for th in ths:
        th.start()
    for th in ths:
        th.join(120)
    batches, requests = b.stats()
    b.close()
    assert not errors, errors
    for k in range(2):
        assert np.array_equal(got[k], want[k]), k
    assert requests == 2 * n and batches < requests


def test_native_batcher_close_while_waiting(engine):
    """hg_batcher_destroy verifies every queued ticket before it returns and
    tickets hold their own state: threads blocked in wait while another thread
    closes the batcher, and waits made after the close, all get their verdicts;
    a submit after the close is refused."""
    import threading

    import bench
    from handel_amd.engine import Batcher, HandelGPUError

    assert engine.set_message(bench.LIB_MESSAGE) == 0
    reqs, words, sigs, expect, _, _ = bench.make_aggregate_batch(engine, 300, 48, seed=37)
    b = Batcher(engine, max_batch=16, max_wait_us=20000)  # a long linger: the close finds tickets queued
    tickets = []
    for i in range(len(reqs)):
        r = reqs[i]
        nw = (int(r["bitlen"]) + 63) // 64
        tickets.append(b.submit(bench.LIB_MESSAGE, int(r["offset"]), int(r["bitlen"]), int(r["level_size"]),
                                words[int(r["word_offset"]):int(r["word_offset"]) + nw], sigs[64 * i:64 * i + 64]))
    got = np.full(len(reqs), -1, dtype=np.int32)

    def waiter(k):
        for i in range(k, 24, 4):
            got[i] = b.wait(tickets[i])

    ths = [threading.Thread(target=waiter, args=(k,)) for k in range(4)]
    for th in ths:
        th.start()
    b.close()  # while the waiters block
    for i in range(24, len(reqs)):  # collected after the batcher is gone
        got[i] = b.wait(tickets[i])
    for th in ths:
        th.join(60)
    assert np.array_equal(got, expect)
    with pytest.raises(HandelGPUError):
        b.submit(bench.LIB_MESSAGE, 0, 0, 1, np.zeros(0, dtype=np.uint64), bytes(64))
