"""CPU suite: the N>1 path (sharding + verdict-bitset gather) with world_size
2 over gloo, and the host logic it relies on."""

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from handel_amd.distributed import gather_verdicts, pack_verdicts, shard_range, unpack_verdicts, verify_sharded


def test_shard_range_covers_batch():
    for n in (1, 7, 4096, 4097):
        for world in (1, 2, 3, 8):
            spans = [shard_range(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            assert max(h - l for l, h in spans) - min(h - l for l, h in spans) <= 1


def test_pack_unpack_roundtrip():
    codes = torch.tensor([0, 1, 0, 0, 2, 0, 0, 0, 1, 0, 0], dtype=torch.int32)
    bits = pack_verdicts(codes)
    assert bits.dtype == torch.uint8 and bits.numel() == 2
    assert bits[0].item() == 0b11101101
    assert torch.equal(unpack_verdicts(bits, 11), codes == 0)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n = 4096
    lo, hi = shard_range(n, rank, world)
    # each rank "verifies" its slice: every 8th check of the global batch invalid
    codes = torch.tensor([1 if i % 8 == 0 else 0 for i in range(lo, hi)], dtype=torch.int32)
    got = gather_verdicts(pack_verdicts(codes), world)
    full = torch.cat([unpack_verdicts(g, hi - lo) for g in got])
    q.put((rank, full.sum().item(), full.numel()))
    dist.destroy_process_group()


def test_two_rank_gloo_gather():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    res = sorted(q.get(timeout=10) for _ in range(world))
    for rank, valid, total in res:
        assert total == 4096 and valid == 4096 - 512


def _pattern(i: int) -> int:
    """A verdict code that depends on the global check index (rank-distinct
    slices get distinct patterns, so a misordered gather shows)."""
    return 0 if (i * 2654435761) % 7 < 4 else 1 + i % 3


def _sharded_worker(rank, world, port, n, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    seen = []

    def verify(lo, hi):
        seen.append((lo, hi))
        return torch.tensor([_pattern(i) for i in range(lo, hi)], dtype=torch.int32)

    full = verify_sharded(verify, n, rank, world, device=torch.device("cpu"))
    q.put((rank, seen, full.tolist()))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 4096), (3, 4097), (3, 5)])
def test_sharded_gather_order(world, n):
    """verify_sharded at world 2 and 3 over gloo: every rank verifies exactly
    its contiguous slice, and every rank ends with the whole batch's verdicts
    in batch order (uneven slices included)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sharded_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    res = sorted(q.get(timeout=10) for _ in range(world))
    want = [_pattern(i) == 0 for i in range(n)]
    for rank, seen, full in res:
        assert seen == [shard_range(n, rank, world)]
        assert full == want
