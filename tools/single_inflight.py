#!/usr/bin/env python3
"""Config 2 (independent single-signature checks, batch 4096) one batch at a
time and with K batches in flight, each in flight batch on a context of its
own (own stream and workspace), every verdict checked.

  HG_VERIFY_SPLIT=0|1 python tools/single_inflight.py OUT.json [K ...]

Prints and writes {K: {ms_per_batch, value}}; the split form
(launch_verify_split) is chosen by HG_VERIFY_SPLIT in the environment.
"""

import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from handel_amd.engine import Engine  # noqa: E402


def main():
    out = sys.argv[1]
    ks = [int(x) for x in sys.argv[2:]] or [1, 2, 4]
    n, steps = 4096, 40
    dev = torch.device("cuda:0")
    kmax = max(ks)
    engs, work = [], []
    for i in range(kmax):
        e = Engine(device=0, flavor="go")
        assert e.set_message(bench.LIB_MESSAGE) == 0
        pks, sigs, expect = bench.make_batch(e, n, seed=1234 + i)
        s = torch.cuda.Stream(dev)
        work.append(dict(pks=bench._dev_bytes(pks, dev), sigs=bench._dev_bytes(sigs, dev),
                         codes=torch.zeros(n, dtype=torch.int32, device=dev), expect=expect, stream=s))
        engs.append(e)
    res = {"split": os.environ.get("HG_VERIFY_SPLIT", "0"), "n": n, "steps": steps}
    for k in ks:
        def submit(j):
            w = work[j]
            engs[j].verify_batch_device(w["pks"].data_ptr(), w["sigs"].data_ptr(), n, w["codes"].data_ptr(),
                                        w["stream"].cuda_stream)
        for j in range(k):
            work[j]["codes"].fill_(-1)
        torch.cuda.synchronize()  # the fills (current stream) before the lanes' streams
        for j in range(k):  # warm-up and parity
            submit(j)
        torch.cuda.synchronize()
        for j in range(k):
            got = work[j]["codes"].cpu().numpy()
            bad = np.flatnonzero(got != work[j]["expect"])
            assert bad.size == 0, f"K={k} lane {j}: verdicts differ at {bad[:8]}: {got[bad[:8]]}"
        t0 = time.perf_counter()
        for it in range(steps):
            submit(it % k)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        res[str(k)] = {"ms_per_batch": round(dt / steps * 1e3, 4), "value": round(n * steps / dt, 1)}
        print(k, res[str(k)], flush=True)
    with open(out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
