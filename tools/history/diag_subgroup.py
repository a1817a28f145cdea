#!/usr/bin/env python3
"""Timing of the registry load, the asynchronous G2 membership check and the
table build (diagnostic tooling)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from handel_amd.engine import Engine  # noqa: E402

torch.cuda.set_device(0)
out = {}
e = Engine(0, "go")
assert e.set_message(bench.LIB_MESSAGE) == 0
reg = e.keygen(bench.seeded_scalars(4000, 1))
for trial in range(3):
    e.sync()
    t0 = time.perf_counter()
    assert not e.registry_load(reg).any()
    t1 = time.perf_counter()
    time.sleep(0.2)
    t2 = time.perf_counter()
    ng = e.registry_non_g2()
    t3 = time.perf_counter()
    assert e.prepare_aggregate() == 0
    t4 = time.perf_counter()
    out[trial] = {"load_ms": (t1 - t0) * 1e3, "non_g2_ms_after_200ms": (t3 - t2) * 1e3, "prepare_ms": (t4 - t3) * 1e3,
                  "non_g2": ng}
e2 = Engine(0, "go")
assert e2.set_message(bench.LIB_MESSAGE) == 0
t0 = time.perf_counter()
assert not e2.registry_load(reg).any()
t1 = time.perf_counter()
ng = e2.registry_non_g2()
t2 = time.perf_counter()
out["immediate"] = {"load_ms": (t1 - t0) * 1e3, "non_g2_wait_ms": (t2 - t1) * 1e3}
print(json.dumps(out))
