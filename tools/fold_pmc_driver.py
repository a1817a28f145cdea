#!/usr/bin/env python3
"""Program for PMC passes over the GT fold alone: the full-registry batch
(4096 requests spanning a 4000-key registry), fold before the pairing
(overlap off), 10 submissions after 3 warm ones (tools/gpu_fold_pmc.sh)."""
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
e.set_fold_overlap(False)
w = bench.AggregateWorkload(e, 4000, 4096, seed=8765, dev=dev, stream=stream, full=True)
for _ in range(13):
    w.submit()
torch.cuda.synchronize(dev)
w.check()
e.close()
print("ok")
