#!/usr/bin/env python3
"""A/B helper for the GT fold's chunk size (HG_GT_CHUNK, read at context
creation): the full-registry workload of bench.py (4096 requests spanning a
4000-key registry, ~250 window terms each) and the headline workload, one
batch at a time and four in flight on unpadded lanes. Prints one JSON line.

  HG_GT_CHUNK=16 python tools/fold_chunk_ab.py
"""

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from handel_amd.engine import Engine  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    stream = torch.cuda.current_stream(dev)
    timer = bench.Timer(dev, False, dev, 1)
    eng = Engine(device=0, flavor="go")
    assert eng.set_message(bench.LIB_MESSAGE) == 0
    out = {"chunk": os.environ.get("HG_GT_CHUNK", "default")}
    for name, full in (("headline", False), ("full_registry", True)):
        wl = bench.AggregateWorkload(eng, 4000, 4096, seed=8765 if full else 4321, dev=dev, stream=stream, full=full)
        dt = timer.run(wl.submit, 30, 5)
        wl.check()
        ph = bench.timed_phases(eng, lambda: [wl.submit() for _ in range(5)])
        eng.set_fold_overlap(False)
        ph_seq = bench.timed_phases(eng, lambda: [wl.submit() for _ in range(5)])
        eng.set_fold_overlap(True)
        idt = bench.lanes_rate(eng, wl, 4, timer, 30, 5, dev)
        out[name] = {"sequential": round(4096 * 30 / dt, 1), "inflight4": round(4096 * 30 / idt, 1),
                     "fold_alone_ms": round(ph_seq["fold"], 4), "fold_beside_ms": round(ph["fold"], 4),
                     "terms": wl.terms}
    print(json.dumps(out))
    eng.close()


if __name__ == "__main__":
    main()
