"""The built gfx950 code objects keep the register and LDS budgets the
kernels' occupancy arguments rest on: no VGPR spills
or scratch in the pairing and fold kernels, the padded pairing kernels above
half the VGPR file (one wave per SIMD), the unpadded 12-lane kernel within it
(two per SIMD), and the LDS sizes the per-CU packing assumes. Reads the
library's metadata notes; no GPU needed (skipped when the library is not
built)."""

import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
LIB = os.path.join(ROOT, "handel_amd", "_build", "libhandel_gpu.so")


@pytest.fixture(scope="module")
def res():
    if not os.path.exists(LIB):
        pytest.skip("libhandel_gpu.so not built")
    import kernel_sizes

    r = kernel_sizes.resources(LIB)
    if not r:
        pytest.skip("no gfx950 code object metadata found")
    return r


def _one(res, part):
    hits = {k: v for k, v in res.items() if part in k}
    assert len(hits) == 1, (part, sorted(hits))
    return next(iter(hits.values()))


HOT = {
    # mangled-name fragment: (LDS bytes, VGPR rule)
    "k_verify_sig12ILb0E": (18400, "two_per_simd"),   # the headline's unpadded 12-lane kernel
    "k_verify_sig12ILb1E": (18400, "padded"),
    "k_sig12_millerILb0E": (18400, "two_per_simd"),   # the split form's two halves (the default)
    "k_sig12_feILb0E": (18400, "two_per_simd"),
    "k_sig12_ninv": (20480, None),
    "k_sig12_norm": (18400, "two_per_simd"),          # config 2's split form: the norm of a given f
    "k_verify_mlILi4E": (20480, "two_per_simd"),      # ... and its Miller loop on layout V (eight waves per CU)
    "k_verify_sigILi4ELb1ELb1E": (18880, "padded"),   # k_verify_sig<4, true, true>: sequential / latency
    "k_verify_sig_splitILi2E": (30144, "padded"),     # the two-wave latency form
    "k_gt_chunks": (12000, None),
    "k_gt_combine": (9600, None),
}


@pytest.mark.parametrize("part", sorted(HOT))
def test_hot_kernels_keep_their_budgets(res, part):
    r = _one(res, part)
    lds, rule = HOT[part]
    assert r["vgpr_spill"] == 0 and r["sgpr_spill"] == 0 and r["scratch"] == 0, (part, r)
    assert r["lds"] == lds, (part, r)
    if rule == "padded":
        assert r["vgpr"] > 256, (part, r)   # > half of the 512-entry file: one wave per SIMD
    elif rule == "two_per_simd":
        assert r["vgpr"] <= 256, (part, r)
