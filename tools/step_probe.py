#!/usr/bin/env python3
"""Where the headline step's time goes beyond the kernels: host time of K
step() calls (no synchronisation) against the GPU time of the same K steps,
for the submission alone, + the verdict pack, + the world-1 gather copy.

  python tools/step_probe.py [steps]
"""

import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from handel_amd.distributed import gather_verdicts  # noqa: E402
from handel_amd.engine import Engine  # noqa: E402


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    stream = torch.cuda.current_stream(dev)
    eng = Engine(device=0, flavor="go")
    assert eng.set_message(bench.LIB_MESSAGE) == 0
    head = bench.AggregateWorkload(eng, 4000, 4096, seed=4321, dev=dev, stream=stream)
    gathered = [torch.zeros(512, dtype=torch.uint8, device=dev)]
    variants = {
        "submit": lambda: head.submit(),
        "submit+pack": lambda: (head.submit(), head.pack()),
        "submit_bits": lambda: head.submit_bits(),
        "submit_bits+gather": lambda: (head.submit_bits(), gather_verdicts(head.d_bits, 1, gathered)),
    }
    out = {}
    for name, fn in variants.items():
        for _ in range(3):
            fn()
        torch.cuda.synchronize(dev)
        best = None
        for _rep in range(3):
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for _ in range(k):
                fn()
            t_host = time.perf_counter() - t0
            torch.cuda.synchronize(dev)
            t_all = time.perf_counter() - t0
            r = {"host_us_per_step": round(t_host / k * 1e6, 1), "ms_per_step": round(t_all / k * 1e3, 4)}
            if best is None or r["ms_per_step"] < best["ms_per_step"]:
                best = r
        out[name] = best
    head.check()
    print(json.dumps(out))
    eng.close()


if __name__ == "__main__":
    main()
