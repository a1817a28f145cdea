#!/usr/bin/env python3
"""Fold-alone and whole-submission times (HIP events) of the headline and the
full-registry batches under the current HG_GT_CHUNK / HG_GT_GRID; one JSON
line (tooling for schedule sweeps)."""
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
e = Engine(0, "go")
assert e.set_message(bench.LIB_MESSAGE) == 0
out = {"chunk": os.environ.get("HG_GT_CHUNK"), "grid": os.environ.get("HG_GT_GRID")}
for name, full in (("headline", False), ("full", True)):
    w = bench.AggregateWorkload(e, 4000, 4096, seed=8765 if full else 4321, dev=dev, stream=stream, full=full)
    for _ in range(3):
        w.submit()
    torch.cuda.synchronize(dev)
    w.check()
    for ov in (False, True):
        e.set_fold_overlap(ov)
        ph = bench.timed_phases(e, lambda: [w.submit() for _ in range(10)])
        out[f"{name}_{'ovl' if ov else 'seq'}"] = {k: round(v, 4) for k, v in ph.items()}
    w.check()
print(json.dumps(out))
