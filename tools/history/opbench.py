#!/usr/bin/env python3
"""Per-building-block cost of the team Fp12 ops (hg_debug_fp12 with reps):
cycles per op per wave = (t(reps=R) - t(reps=1)) / (R - 1) at 4096 elements
(1024 single-wave blocks = one wave per SIMD, like k_verify). Diagnostic tool."""

import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from handel_amd.engine import Engine  # noqa: E402

P = 65000549695646603732796438742359905742825358107623003571877145026864184071783
NAMES = {0: "mul", 1: "sqr_fast", 2: "cyc_sqr", 3: "frob", 4: "frob2", 5: "inv", 6: "conj",
         9: "sqr_table", 10: "cyc_sqr_table"}


def main():
    eng = Engine(0, "go")
    n = 4096
    rng = np.random.default_rng(1)
    a = b"".join(b"".join((int.from_bytes(rng.bytes(32), "big") % P).to_bytes(32, "big") for _ in range(12))
                 for _ in range(n))
    res = {}
    R = 41
    for op, name in NAMES.items():
        ts = []
        for reps in (1, R):
            eng.fp12_op(op | (reps << 8), a, a)  # warm
            t0 = time.perf_counter()
            for _ in range(3):
                eng.fp12_op(op | (reps << 8), a, a)
            ts.append((time.perf_counter() - t0) / 3)
        per_op_us = (ts[1] - ts[0]) / (R - 1) * 1e6
        res[name] = {"us_per_op": round(per_op_us, 3), "cycles_per_op_at_2.4GHz": round(per_op_us * 2400)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
