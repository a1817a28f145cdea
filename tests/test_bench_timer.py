"""bench.Timer across ranks (gloo, world 2, CPU): the prewarm runs the same
number of steps on every rank even when the ranks' steps take different
times (each step holds a collective, as bench.py's headline step holds the
verdict gather), and run() reports the max over ranks."""

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, q):
    import time

    import bench

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cpu = torch.device("cpu")
        t = bench.Timer(cpu, True, cpu, world)

        def step():  # rank 1 is 3x slower; every step gathers
            time.sleep(0.002 * (1 + 2 * rank))
            out = [torch.zeros(1) for _ in range(world)]
            dist.all_gather(out, torch.ones(1) * rank)

        k = t.prewarm(step, 0.15)
        dt = t.run(step, 5, 2)
        q.put((rank, k, dt, t.rank_times))
    finally:
        dist.destroy_process_group()


def test_prewarm_agrees_across_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    (_, k0, dt0, rt0), (_, k1, dt1, rt1) = res
    assert k0 == k1 > 1
    assert dt0 == dt1 == max(rt0) and len(rt0) == 2
