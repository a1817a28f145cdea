"""GPU suite: the N > 1 path through the real engine.

Two ranks (torch.distributed over gloo, both on the one GPU of the test box:
the production launch is one rank per GPU over RCCL) each verify their
contiguous slice of one config-3 batch through hg_verify_aggregate (the GT
path) and all-gather the verdict bitsets (handel_amd.distributed.verify_sharded).
Every rank must end with the whole batch's verdicts, in batch order, equal to
the expected pattern (1/8 tampered) — the only cross-rank traffic is the
bitset gather.
"""

import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, q):
    import sys

    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist

    import bench
    from handel_amd.distributed import shard_range, verify_sharded
    from handel_amd.engine import Engine

    dist.init_process_group("gloo", rank=rank, world_size=world)
    eng = Engine(device=0, flavor="go")
    eng.set_aggregate_level(2)  # the GT path whatever the volume
    try:
        assert eng.set_message(bench.LIB_MESSAGE) == 0
        # every rank builds the same batch (same seed) and verifies its slice
        reqs, words, sigs, expect, _, _ = bench.make_aggregate_batch(eng, 500, 600, seed=21)
        seen = []

        def verify(lo, hi):
            seen.append((lo, hi))
            codes = eng.verify_aggregate(reqs[lo:hi], words, sigs[64 * lo:64 * hi])
            return torch.from_numpy(np.asarray(codes, dtype=np.int32))

        full = verify_sharded(verify, len(reqs), rank, world, device=torch.device("cpu"))
        q.put((rank, seen, full.tolist(), [bool(c == 0) for c in expect], shard_range(len(reqs), rank, world)))
    finally:
        eng.close()
        dist.destroy_process_group()


def test_two_ranks_verify_and_gather():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
        assert p.exitcode == 0
    res = sorted(q.get(timeout=10) for _ in range(world))
    for rank, seen, full, want, span in res:
        assert seen == [span]
        assert full == want
        assert sum(want) < len(want)  # the tampered eighth is in there


def _committee_rank(rank, world, port, q):
    """Config 5: rank r is committee r — its OWN 4096-key registry (rank-seeded)
    and its own 512 multisigs, one extra tampered aggregate at a rank-distinct
    position; the ranks all-gather their verdict bitsets."""
    import sys

    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist

    import bench
    from handel_amd.distributed import gather_verdicts, pack_verdicts
    from handel_amd.engine import Engine

    dist.init_process_group("gloo", rank=rank, world_size=world)
    eng = Engine(device=0, flavor="go")
    eng.set_aggregate_level(2)
    try:
        assert eng.set_message(bench.LIB_MESSAGE) == 0
        reqs, words, sigs, expect, _, reg = bench.make_aggregate_batch(eng, 4096, 512, seed=300 + rank)
        j = 8 * rank + 3  # rank-distinct extra tamper (not on the every-8th grid)
        bad, _ = eng.combine_g1(sigs[64 * j:64 * j + 64], bench.G1_GEN_BYTES)
        sigs = sigs[:64 * j] + bad + sigs[64 * j + 64:]
        expect = expect.copy()
        expect[j] = 1
        assert eng.prepare_aggregate() == 0
        codes = torch.from_numpy(np.asarray(eng.verify_aggregate(reqs, words, sigs), dtype=np.int32))
        out = gather_verdicts(pack_verdicts(codes), world)
        q.put((rank, [o.tolist() for o in out], pack_verdicts(torch.from_numpy(expect)).tolist(),
               reg[:128].hex()))
    finally:
        eng.close()
        dist.destroy_process_group()


def test_committees_one_registry_per_rank():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_committee_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
        assert p.exitcode == 0
    res = sorted(q.get(timeout=10) for _ in range(world))
    expects = [e for _, _, e, _ in res]
    assert expects[0] != expects[1]              # the committees' verdict patterns differ
    assert res[0][3] != res[1][3]                # and so do their registries
    for rank, gathered, _, _ in res:
        assert gathered == expects               # every rank holds every committee's verdicts, in rank order
