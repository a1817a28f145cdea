#!/usr/bin/env python3
"""Times the signature-pairing kernels alone (hg_sig_pairing_device) on a
4096-signature batch: kernel 2 (12-lane, padded: one wave per SIMD) once at a
time, and kernel 3 (12-lane, unpadded) with four launches in flight on four
streams (the headline's regime). HG_LIB picks the library (A/B of variants).
Prints one JSON line. Values are not checked (probe variants may be wrong)."""

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from handel_amd.engine import Engine  # noqa: E402


def main():
    n = 4096
    eng = Engine(device=0, flavor="go")
    assert eng.set_message(bench.LIB_MESSAGE) == 0
    kb = bench.seeded_scalars(n, 77)
    sigs = eng.sign(kb)
    dev = torch.device("cuda", 0)
    d_sigs = torch.frombuffer(bytearray(sigs), dtype=torch.uint8).to(dev)
    out = {"lib": os.environ.get("HG_LIB", "default")}
    for kernel, flight in ((2, 1), (3, 4)):
        streams = [torch.cuda.Stream(dev) for _ in range(flight)]
        engs = [eng] + [Engine(device=0, flavor="go") for _ in range(flight - 1)]
        fes = [torch.empty(n * 480, dtype=torch.uint8, device=dev) for _ in range(flight)]
        for e in engs[1:]:
            assert e.set_message(bench.LIB_MESSAGE) == 0

        def step(i):
            engs[i % flight].sig_pairing_device(d_sigs.data_ptr(), n, fes[i % flight].data_ptr(), kernel,
                                                streams[i % flight].cuda_stream)

        for i in range(2 * flight):
            step(i)
        torch.cuda.synchronize(dev)
        reps = 40
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record(torch.cuda.current_stream(dev))
        for s in streams:
            s.wait_stream(torch.cuda.current_stream(dev))
        for i in range(reps):
            step(i)
        for s in streams:
            torch.cuda.current_stream(dev).wait_stream(s)
        ev[1].record(torch.cuda.current_stream(dev))
        torch.cuda.synchronize(dev)
        ms = ev[0].elapsed_time(ev[1]) / reps
        out[f"kernel{kernel}_inflight{flight}_ms_per_batch"] = round(ms, 4)
        out[f"kernel{kernel}_inflight{flight}_checks_per_s"] = round(n / ms * 1e3, 1)
        for e in engs[1:]:
            e.close()
    eng.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
