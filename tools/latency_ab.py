#!/usr/bin/env python3
"""A/B helper for the per-batch latency floor: bench.py's batch_latency
(one batch of n headline requests submitted alone and waited for) and,
unless --no-proxy, the config-4 proxy's service line. The pairing kernel
choice comes from the environment (HG_SIG_W2=0: the one-wave k_verify_sig).
Prints one JSON line.

  HG_SIG_W2=0 python tools/latency_ab.py
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
    eng = Engine(device=0, flavor="go")
    assert eng.set_message(bench.LIB_MESSAGE) == 0
    head = bench.AggregateWorkload(eng, 4000, 4096, seed=4321, dev=dev, stream=stream)
    out = {"HG_SIG_W2": os.environ.get("HG_SIG_W2", "default")}
    if "--no-check" not in sys.argv:  # (--no-check: kernel times only, for timing-probe builds)
        bench.batch_latency(eng, head, dev, sizes=(32, 128), reps=5)  # warm
        out["batch_latency"] = bench.batch_latency(eng, head, dev, sizes=(1, 32, 128, 512, 2048, 4096), reps=25)
    # the pairing kernels alone (HIP events on one stream): the one-wave
    # k_verify_sig and the two-wave k_verify_sig_split<2>, by batch size
    out["kernel_ms"] = {}
    ks = torch.cuda.Stream(dev)  # the events and the launches on one stream
    for n in (128, 1024, 2048):
        fe = torch.empty(n * 480, dtype=torch.uint8, device=dev)
        row = {}
        for k, name in ((Engine.SIG_K16_PAD, "k_verify_sig"), (Engine.SIG_W2, "k_verify_sig_split<2>")):
            for _ in range(2):
                eng.sig_pairing_device(head.d_sigs.data_ptr(), n, fe.data_ptr(), k, ks.cuda_stream)
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record(ks)
            for _ in range(10):
                eng.sig_pairing_device(head.d_sigs.data_ptr(), n, fe.data_ptr(), k, ks.cuda_stream)
            ev[1].record(ks)
            torch.cuda.synchronize(dev)
            row[name] = round(ev[0].elapsed_time(ev[1]) / 10, 4)
        out["kernel_ms"][str(n)] = row
    eng.close()
    if "--no-proxy" not in sys.argv:
        out["config4_service"] = bench.config4_proxy("service")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
