#!/usr/bin/env python3
"""A/B on one box: fold beside the pairing kernel (overlap) vs before it, for
the headline batch, two batches in flight (two contexts, two streams) and the
full-registry batch. Prints one JSON line. Tooling, not the bench."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from handel_amd.engine import Engine  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
stream = torch.cuda.current_stream(dev)
timer = bench.Timer(dev, False, dev)
steps, warm, n = 30, 5, 4096
out = {}
engs = [Engine(0, "go") for _ in range(2)]
for e in engs:
    assert e.set_message(bench.LIB_MESSAGE) == 0
head = bench.AggregateWorkload(engs[0], 4000, n, seed=4321, dev=dev, stream=stream)
assert not engs[1].registry_load(head.reg).any() and engs[1].prepare_aggregate() == 0
st2 = torch.cuda.Stream(dev)
c2 = torch.zeros(n, dtype=torch.int32, device=dev)
for ov in (True, False):
    for e in engs:
        e.set_fold_overlap(ov)
    dt = timer.run(head.submit, steps, warm)
    head.check()
    dtp = timer.run(lambda: (head.submit(), head.submit(eng=engs[1], codes=c2, stream=st2)), steps, warm)
    head.check(c2)
    out["overlap" if ov else "sequential"] = {"headline": round(n * steps / dt, 1),
                                              "pipelined2": round(2 * n * steps / dtp, 1)}
full = bench.AggregateWorkload(engs[0], 4000, n, seed=8765, dev=dev, stream=stream, full=True)
for ov in (True, False):
    engs[0].set_fold_overlap(ov)
    dt = timer.run(full.submit, steps, warm)
    full.check()
    out["overlap" if ov else "sequential"]["full_registry"] = round(n * steps / dt, 1)
print(json.dumps(out))
