"""CPU suite: the product's variable-time Bernstein-Yang inversion
(handel_amd/csrc/bn256_inv.h, behind fp_inv) compiled for the host and checked
against Python's pow(a, -1, p) — the value x/crypto's gfP.Invert (a^(p-2))
returns — on edge cases and random field elements."""

import os
import random
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = 65000549695646603732796438742359905742825358107623003571877145026864184071783


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("inv") / "inv_harness")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "handel_amd", "csrc"),
                           os.path.join(ROOT, "tests", "native", "inv_harness.cpp"), "-o", exe])
    return exe


def run(exe, vals, use62=False):
    inp = "".join(" ".join("%x" % ((v >> (32 * i)) & 0xFFFFFFFF) for i in range(8)) + "\n" for v in vals)
    out = subprocess.run([exe] + (["62"] if use62 else []), input=inp, capture_output=True, text=True,
                         check=True).stdout.split("\n")
    return [sum(int(x, 16) << (32 * i) for i, x in enumerate(line.split())) for line in out[:len(vals)]]


def test_constants():
    import re

    src = open(os.path.join(ROOT, "handel_amd", "csrc", "bn256_inv.h")).read()
    limbs = [int(x, 16) for x in re.search(r"#define HG_P62 (.*)", src).group(1).replace("ll", "").split(",")]
    assert sum(l << (62 * i) for i, l in enumerate(limbs)) == P
    inv = int(re.search(r"kPInv62 = (0x[0-9a-f]+)ull", src).group(1), 16)
    assert (P * inv) % (1 << 62) == 1
    limbs = [int(x, 16) for x in re.search(r"#define HG_P30 (.*)", src).group(1).split(",")]
    assert sum(l << (30 * i) for i, l in enumerate(limbs)) == P and all(l < (1 << 30) for l in limbs)
    inv = int(re.search(r"kPInv30 = (0x[0-9a-f]+)u", src).group(1), 16)
    assert (P * inv) % (1 << 30) == 1


@pytest.mark.parametrize("use62", [False, True], ids=["signed30", "signed62"])
def test_inverse_matches_fermat(harness, use62):
    rng = random.Random(5)
    vals = [0, 1, 2, 3, P - 1, P - 2, (P - 1) // 2, 1 << 255, (1 << 200) + 1, 2**62, 2**62 - 1]
    vals += [rng.randrange(P) for _ in range(5000)]
    vals += [rng.randrange(1 << 64) for _ in range(200)]  # short inputs (early length reduction)
    got = run(harness, vals, use62)
    for v, r in zip(vals, got):
        assert r == (pow(v, P - 2, P)), v
