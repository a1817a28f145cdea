#!/usr/bin/env python3
"""Sweep for the full-registry workload with batches in flight (bench.py's
full_registry.inflight line: 4096 requests spanning a 4000-key registry,
~220 window terms each): lanes in flight x padded/unpadded pairing kernel x
fold beside the pairing (overlap) or before it. Kernel choice otherwise from
the environment (HG_SIG12). Prints one JSON line.

  python tools/full_inflight_ab.py
"""

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from handel_amd.engine import DeviceLane, Engine  # noqa: E402


def rate(eng, wl, inflight, pad, overlap, timer, steps, warmup, dev):
    lanes = [DeviceLane(eng, wl.n, pad=pad, overlap=overlap) for _ in range(inflight)]
    codes = [torch.zeros(wl.n, dtype=torch.int32, device=dev) for _ in lanes]
    turn = [0]

    def st():
        i = turn[0] % inflight
        turn[0] += 1
        lanes[i].submit_device(wl.d_reqs.data_ptr(), wl.n, wl.d_words.data_ptr(), wl.d_sigs.data_ptr(),
                               codes[i].data_ptr(), 0, lanes[i].stream)

    try:
        for _ in range(inflight):
            st()
        torch.cuda.synchronize(dev)
        dt = timer.run(st, steps, warmup)
        for c in codes:
            wl.check(c)
    finally:
        for ln in lanes:
            ln.close()
    return round(wl.n * steps / dt, 1)


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    stream = torch.cuda.current_stream(dev)
    timer = bench.Timer(dev, False, dev, 1)
    eng = Engine(device=0, flavor="go")
    assert eng.set_message(bench.LIB_MESSAGE) == 0
    wl = bench.AggregateWorkload(eng, 4000, 4096, seed=8765, dev=dev, stream=stream, full=True)
    out = {"HG_SIG12": os.environ.get("HG_SIG12", "auto"), "terms": wl.terms}
    for overlap in (True, False):
        for pad in (False, True):
            for inflight in (2, 3, 4, 6):
                key = f"{'overlap' if overlap else 'serial'}_{'pad' if pad else 'unpad'}_{inflight}"
                out[key] = rate(eng, wl, inflight, pad, overlap, timer, 30, 6, dev)
                print(key, out[key], file=sys.stderr, flush=True)
    print(json.dumps(out))
    eng.close()


if __name__ == "__main__":
    main()
