"""tools/busy_summary.py: the per-step device-busy time behind bench.py's
frac_rocprof. Synthetic kernel rows: overlapping kernels
merge, kernels partly outside the timed region are clipped, and the clock
whose window holds the kernels is the one used."""

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import busy_summary as B  # noqa: E402


def test_union_merges_overlaps():
    assert B.union_ns([(0, 10), (5, 15), (20, 30)]) == 25
    assert B.union_ns([(0, 10), (2, 3), (10, 12)]) == 12
    assert B.union_ns([]) == 0


def test_summary_clips_to_the_timed_region_and_picks_the_clock():
    rows = [("void hg::k_a<false>(int)", 900, 1100),   # starts before the region: clipped to 1000
            ("hg::k_b(int)", 1050, 1400),               # overlaps k_a
            ("hg::k_b(int)", 1500, 1700),
            ("hg::k_c(int)", 1900, 2300)]               # ends after the region: clipped to 2000
    marks = {"monotonic": [1000, 2000], "realtime": [10 ** 18, 10 ** 18 + 1000]}
    r = B.summarise(rows, marks, steps=2)
    assert r["clock"] == "monotonic" and r["kernels"] == 4
    # busy: [1000, 1400) + [1500, 1700) + [1900, 2000) = 700 ns over 2 steps
    assert r["busy_ms_per_step"] == round(700 / 1e6 / 2, 4)
    assert r["window_ms_per_step"] == round(1000 / 1e6 / 2, 4)
    assert abs(r["idle_fraction"] - 0.3) < 1e-9
    assert r["per_kernel"]["hg::k_b"]["dispatches_per_step"] == 1.0
