#!/usr/bin/env python3
"""Phase breakdown of the pairing-check kernel from the diagnostic build
(-DHG_DIAG, in-kernel s_memtime counters; never the timed product build).

Usage: python tools/diag.py            (builds libhandel_gpu_diag.so if needed)
Prints one JSON line: mean cycles per block (one wave = 4 checks) per phase.
"""

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from handel_amd import build as B  # noqa: E402

os.environ["HG_LIB"] = B.build_library(diag=True)

import numpy as np  # noqa: E402

import bench  # noqa: E402
from handel_amd.engine import Engine  # noqa: E402

NAMES = ["fixed_line_load", "mdbl1_sqr_and_dbl_r1", "mdbl2_fixline_and_dbl_r2", "pk_line_mul", "add_step", "fe_inversion", "fe_rest",
         "fe_pow_u_x3", "miller_total", "final_exp_total", "kernel_total"]


def main():
    eng = Engine(0, "go")
    assert eng.set_message(bench.LIB_MESSAGE) == 0
    n = 4096
    pks, sigs, expect = bench.make_batch(eng, n, seed=7)
    codes = eng.verify_batch(pks, sigs)
    assert np.array_equal(codes, expect)
    out = np.zeros(4096 * 16, dtype=np.uint64)
    rc = eng.L.hg_diag_read(eng.ctx, out.ctypes.data, out.size)
    assert rc == 0, "not a diagnostic build"
    blocks = n // 4
    d = out.reshape(4096, 16)[:blocks].astype(np.float64)
    res = {name: round(float(d[:, i].mean())) for i, name in enumerate(NAMES)}
    res["blocks"] = blocks
    print(json.dumps(res))


if __name__ == "__main__":
    main()
