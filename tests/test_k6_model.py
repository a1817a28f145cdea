"""CPU model of the GT fold's 6-lane Fp12 product (handel_amd/csrc/bn256_k6.h).

The HIP kernels k_gt_chunks6 / k_gt_combine6 / k_gt_win16_6 compute every
Fp2 coefficient c_k of A * B (Fp12 = Fp2[w]/(w^6 - xi)) on one lane as two
passes of lazy 64-bit column sums over 26-bit limbs (Karatsuba in Fp2) and two
REDCs. This model restates that arithmetic limb by limb in Python integers,
with the constants read from the header itself (kK6C, kP4L), and checks:
  * every column's exact value lies in [0, 2^64), so the kernel's mod-2^64
    column arithmetic (including the differences T0 + C - T1 and T2 - T0 - T1)
    is exact;
  * every REDC input is below p R (R = 2^286), so REDC returns < 2p and one
    conditional subtraction makes the output canonical;
  * the result equals schoolbook Fp12 multiplication in the w basis over the
    same Montgomery representatives,
for random operands and for the worst case (every limb at its maximum).
The GPU suite (tests/test_gpu_gt.py) checks the kernels' GT values end to end
against the oracle.
"""

import os
import random
import re

import pytest

from oracle.bn256_oracle import P

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "handel_amd", "csrc", "bn256_k6.h")
LB, NL, RS = 26, 10, 11  # limb bits, limbs, REDC digits (R = 2^286)
R = 1 << (LB * RS)
M64 = (1 << 64) - 1


def _array(name):
    src = open(HDR).read()
    body = re.search(name + r"\[\d+\] = \{([^}]*)\}", src).group(1)
    return [int(t.rstrip("ul"), 16) for t in re.findall(r"0x[0-9a-fA-F]+u?l*", body)]


K6C = _array("kK6C")
P4L = _array("kP4L")


def limbs(x):
    return [(x >> (LB * i)) & ((1 << LB) - 1) for i in range(NL)]


def value(ls):
    return sum(v << (LB * i) for i, v in enumerate(ls))


def xi_lazy(x, y):
    """k6_put's X = xi (x i + y): (3x + y, 3y + (4p)'' - x), limb-wise"""
    xl, yl = limbs(x), limbs(y)
    return [3 * a + b for a, b in zip(xl, yl)], [3 * b + q - a for a, b, q in zip(xl, yl, P4L)]


def columns(acc, u, v):
    for i in range(NL):
        for j in range(NL):
            acc[i + j] += u[i] * v[j]


def redc(cols, checks):
    for c in cols:
        assert 0 <= c < (1 << 64), "column overflow"
    v = sum(c << (LB * i) for i, c in enumerate(cols))
    assert v < P * R, "REDC input above p R"
    checks.append(v.bit_length())
    return v * pow(R, -1, P) % P


def lane_coeff(k, A, B, checks):
    """lane k of a team: A, B = six (x, y) pairs of canonical Montgomery reps"""
    Al = [(limbs(x), limbs(y)) for x, y in A]
    Xl = [xi_lazy(x, y) for x, y in A]
    Bl = [(limbs(x), limbs(y)) for x, y in B]
    t0, t1, t2 = [0] * 21, [0] * 21, [0] * 21
    for i in range(6):
        ux, uy = Al[i] if i <= k else Xl[i]
        vx, vy = Bl[(k - i) % 6]
        for lv in ux + uy:
            assert 0 <= lv < 2 ** 28.34
        columns(t0, uy, vy)
        columns(t1, ux, vx)
        columns(t2, [a + b for a, b in zip(ux, uy)], [a + b for a, b in zip(vx, vy)])
    c = K6C + [0, 0]
    # pass 1 columns: T0 + C and T1 (each < 2^64), then re = T0 + C - T1 >= 0
    for j in range(21):
        assert t0[j] + c[j] < (1 << 64) and t1[j] < (1 << 64)
        assert t0[j] + c[j] - t1[j] >= 0, "re column negative"
    re_cols = [t0[j] + c[j] - t1[j] for j in range(21)]
    # pass 2: the accumulator restarts at -(T0 + T1) mod 2^64 and takes T2; the
    # exact column is T2 - T0 - T1 (>= 0: the cross products)
    im_cols = []
    for j in range(21):
        wrapped = ((c[j] - (t0[j] + c[j]) - t1[j]) + t2[j]) & M64
        exact = t2[j] - t0[j] - t1[j]
        assert 0 <= exact < (1 << 64) and wrapped == exact
        assert t2[j] < (1 << 64)
        im_cols.append(exact)
    return redc(im_cols, checks), redc(re_cols, checks)


def f2_mul(a, b):  # (x i + y)(x' i + y'), i^2 = -1
    return ((a[0] * b[1] + a[1] * b[0]) % P, (a[1] * b[1] - a[0] * b[0]) % P)


def f2_xi(a):  # xi = i + 3
    return ((3 * a[0] + a[1]) % P, (3 * a[1] - a[0]) % P)


def schoolbook(A, B):
    out = [(0, 0)] * 6
    for i in range(6):
        for j in range(6):
            t = f2_mul(A[i], B[j])
            if i + j >= 6:
                t = f2_xi(t)
            k = (i + j) % 6
            out[k] = ((out[k][0] + t[0]) % P, (out[k][1] + t[1]) % P)
    rinv = pow(R, -1, P)
    return [(x * rinv % P, y * rinv % P) for x, y in out]


def test_constants_are_multiples_of_p():
    assert len(K6C) == 19 and len(P4L) == 10
    assert value(K6C) % P == 0 and all((1 << 61) <= c < (1 << 61) + (1 << 26) for c in K6C)
    assert value(P4L) == 4 * P and all(v >= (1 << 26) for v in P4L[:9])


@pytest.mark.parametrize("case", ["random", "max", "mixed"])
def test_lane_products_match_schoolbook(case):
    rng = random.Random(case)
    for _ in range(6 if case == "random" else 2):
        if case == "max":
            A = [(P - 1, P - 1)] * 6
            B = [(P - 1, P - 1)] * 6
        elif case == "mixed":
            A = [(P - 1, 0) if i % 2 else (0, P - 1) for i in range(6)]
            B = [(rng.randrange(P), P - 1) for _ in range(6)]
        else:
            A = [(rng.randrange(P), rng.randrange(P)) for _ in range(6)]
            B = [(rng.randrange(P), rng.randrange(P)) for _ in range(6)]
        checks = []
        got = [lane_coeff(k, A, B, checks) for k in range(6)]
        assert got == schoolbook(A, B)
        assert max(checks) <= 530  # the header's bound: REDC inputs < 2^529.1
