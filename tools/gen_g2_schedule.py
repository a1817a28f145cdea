#!/usr/bin/env python3
"""Generates handel_amd/csrc/bn256_g2sched.h: lane-parallel "team programs"
for a 16-lane team (bn256_g2team.h executes them).

A program is a short list of rounds. In a round every lane of the team
computes one Fp element
    dst = sum_{slot} (sum_m ca_m * X[ra_m]) * (sum_m cb_m * X[rb_m])
with small signed integer coefficients and ONE lazy Montgomery reduction,
then stores it; all lanes run the same instruction stream (only addresses
and coefficients differ), rounds are separated by a team barrier (every
lane reads before any lane writes, so in-place programs are fine).

Operand index space (uint8):
    0..127    the team's LDS register file F (Fp elements)
    128..139  element e of the program's Fp12 source slot A (2k + c)
    160..171  element e of the program's Fp12 source slot B
Destination: an F register (< 128), element e of the destination Fp12
slot (128 + e), or 255 (lane idle).

Programs:
    DBL, ADD_*     x/crypto optate.go lineFunctionDouble / lineFunctionAdd
    CYC_SQR        Granger-Scott squaring in the cyclotomic subgroup
                   (final exponentiation: gfP12.Exp(.., u) squarings)
    SQR12          Fp12 squaring with the symmetric products merged
The tables are validated here by interpreting them with plain modular
arithmetic against the oracle (tests/test_g2_schedule.py repeats this in
the CPU suite). Build tooling only: nothing in the product imports it.
"""

from __future__ import annotations

import os
import random
import sys

P = 65000549695646603732796438742359905742825358107623003571877145026864184071783
R_BITS = 286  # Montgomery R = 2^286 (11 REDC digits, bn256_constants.h kRedcSteps)
R_OVER_P = (1 << R_BITS) / P  # REDC(T) < T/R + p
MAX_NSLOT = 7
MAX_TERMS = 6
SLOT_A = 128
SLOT_B = 160
NONE = 255

# ------------------------------------------------------------------ register file
FP_SCALARS = ["ZERO", "ONE", "PX", "PY", "SX", "NSY"]
# The kernels' register file (kG2Regs): the projective Miller-loop programs'
# point, pk, line coefficients and temporaries. FBX, FCY must stay
# consecutive (load_fixed_line: the normalised G2Base line, a = 1).
FP2_RUNTIME = ["X", "Y", "Z", "QX", "QY", "NQY", "P1X", "P1Y", "P2X",
               "FBX", "FCY", "FB", "FC", "LA", "LB", "LC",
               # projective doubling temporaries
               "A", "B", "S", "C", "G",
               # projective addition temporaries
               "AB", "S1", "D", "I", "S2", "H", "J", "AV", "L1"]
# only the Jacobian x/crypto-shaped programs (DBL, ADD_*: generator
# cross-checks, never run by a kernel) use these; they lie past kG2Regs
FP2_LEGACY = ["T", "R2", "P1R2", "F2ONE", "F2ZERO", "W", "V", "ET", "ZP", "TPY", "XN", "YJ", "TP", "LA1", "S3"]
FP2_REGS = FP2_RUNTIME + FP2_LEGACY
REG = {}
for i, n in enumerate(FP_SCALARS):
    REG[n] = i
_base = len(FP_SCALARS)
for i, n in enumerate(FP2_REGS):
    REG[n + ".x"] = _base + 2 * i
    REG[n + ".y"] = _base + 2 * i + 1
NREGS = _base + 2 * len(FP2_REGS)
NREGS_RUNTIME = _base + 2 * len(FP2_RUNTIME)
assert NREGS <= 128
# Fp12 source slots: Fp2 coefficient k of slot A is "A{k}", of slot B "B{k}"
for k in range(6):
    for ci, c in enumerate("xy"):
        REG[f"A{k}.{c}"] = SLOT_A + 2 * k + ci
        REG[f"B{k}.{c}"] = SLOT_B + 2 * k + ci
        REG[f"D{k}.{c}"] = SLOT_A + 2 * k + ci  # destination slot element (same encoding)


def comp(name, c):
    return REG[f"{name}.{c}"]


# ------------------------------------------------------------------ expression helpers
# An Fp2 linear combination is a list of (fp2_name, coef); its component c is
# the Fp lincomb [(reg(name.c), coef)].
def fp2_comp(lc, c):
    return [(comp(n, c), k) for n, k in lc]


def neg(terms):
    return [(r, -k) for r, k in terms]


def scale(terms, s):
    return [(r, k * s) for r, k in terms]


def add(*ts):
    out = {}
    for t in ts:
        for r, k in t:
            out[r] = out.get(r, 0) + k
    return [(r, k) for r, k in out.items() if k != 0] or [(REG["ZERO"], 1)]


def one():
    return [(REG["ONE"], 1)]


def scal(name):
    return [(REG[name], 1)]


class Lane:
    def __init__(self, dst, slots):
        self.dst = dst
        self.slots = slots  # list of (A_terms, B_terms)


def sq(dst, U):
    """dst (Fp2) = U^2 : two lanes (x, y)."""
    ux, uy = fp2_comp(U, "x"), fp2_comp(U, "y")
    return [Lane(comp(dst, "x"), [(add(ux, ux), uy)]),
            Lane(comp(dst, "y"), [(add(uy, ux), add(uy, neg(ux)))])]


def mul(dst, U, V, extra=None):
    """dst (Fp2) = U * V (+ extra * 1, extra an Fp2 lincomb)."""
    ux, uy = fp2_comp(U, "x"), fp2_comp(U, "y")
    vx, vy = fp2_comp(V, "x"), fp2_comp(V, "y")
    lx = Lane(comp(dst, "x"), [(ux, vy), (uy, vx)])
    ly = Lane(comp(dst, "y"), [(uy, vy), (neg(ux), vx)])
    if extra is not None:
        lx.slots.append((fp2_comp(extra, "x"), one()))
        ly.slots.append((fp2_comp(extra, "y"), one()))
    return [lx, ly]


def sq_plus(dst, U, extra):
    lanes = sq(dst, U)
    lanes[0].slots.append((fp2_comp(extra, "x"), one()))
    lanes[1].slots.append((fp2_comp(extra, "y"), one()))
    return lanes


def smul(dst, U, s_name, k=1):
    """dst (Fp2) = k * U * s (s an Fp scalar register)."""
    return [Lane(comp(dst, c), [([(r, kk * k) for r, kk in fp2_comp(U, c)], scal(s_name))]) for c in ("x", "y")]


def lin(dst, U):
    return [Lane(comp(dst, c), [(fp2_comp(U, c), one())]) for c in ("x", "y")]


# Fp-level product terms of Fp2 expressions, for building sums per component.
def prod_terms(U, V, c, k=1):
    """component c of k * U * V as a list of Fp slots."""
    ux, uy = fp2_comp(U, "x"), fp2_comp(U, "y")
    vx, vy = fp2_comp(V, "x"), fp2_comp(V, "y")
    if c == "x":
        return [(scale(ux, k), vy), (scale(uy, k), vx)]
    return [(scale(uy, k), vy), (scale(neg(ux), k), vx)]


def sq_terms(U, c, k=1):
    ux, uy = fp2_comp(U, "x"), fp2_comp(U, "y")
    if c == "x":
        return [(scale(add(ux, ux), k), uy)]
    return [(scale(add(uy, ux), k), add(uy, neg(ux)))]


def xi_terms(slots_x, slots_y, c):
    """component c of xi * Z where Z = (sum slots_x, sum slots_y):
    xi Z = (3 Zx + Zy) i + (3 Zy - Zx)."""
    if c == "x":
        return [(scale(a, 3), b) for a, b in slots_x] + list(slots_y)
    return [(scale(a, 3), b) for a, b in slots_y] + [(neg(a), b) for a, b in slots_x]


# ------------------------------------------------------------------ programs
def fixed_line_eval(sfx=""):
    # FB = FBX * SX, FC = FCY * NSY  (the G2Base line at -sig), line set sfx
    return smul("FB" + sfx, [("FBX" + sfx, 1)], "SX") + smul("FC" + sfx, [("FCY" + sfx, 1)], "NSY")


def prog_double():
    """lineFunctionDouble(r = (X, Y, Z, T), q = (PX, PY)) -> X,Y,Z,T updated; LA, LB, LC."""
    r1 = sq("A", [("X", 1)]) + sq("B", [("Y", 1)]) + sq("S", [("Y", 1), ("Z", 1)]) + fixed_line_eval() \
        + smul("TPY", [("T", 1)], "PY")
    r2 = (sq("C", [("B", 1)]) + sq("W", [("X", 1), ("B", 1)]) + sq("G", [("A", 3)])
          + sq("V", [("X", 1), ("A", 3)]) + mul("ET", [("A", 3)], [("T", 1)])
          + lin("ZP", [("S", 1), ("B", -1), ("T", -1)]))
    # D = 2(W - A - C); X' = G - 2D; Y' = (D - X') E - 8C = (6W - 6A - 6C - G) 3A - 8C
    r3 = (mul("Y", [("W", 6), ("A", -6), ("C", -6), ("G", -1)], [("A", 3)], extra=[("C", -8)])
          + lin("X", [("G", 1), ("W", -4), ("A", 4), ("C", 4)])
          + sq("T", [("ZP", 1)])
          + smul("LB", [("ET", -2)], "PX")
          + mul("LC", [("ZP", 2)], [("TPY", 1)])
          + lin("LA", [("V", 1), ("A", -1), ("G", -1), ("B", -4)])
          + lin("Z", [("ZP", 1)]))
    return [r1, r2, r3]


def prog_add(px, py, pr2):
    """lineFunctionAdd(r = (X,Y,Z,T), p = (px, py), q = (PX, PY), r2 = pr2)."""
    a1 = mul("AB", [(px, 1)], [("T", 1)]) + sq("S1", [(py, 1), ("Z", 1)]) + fixed_line_eval()
    # D = (S1 - r2 - T) T ; H = AB - X ; I = H^2 ; S2 = (Z + H)^2
    a2 = (mul("D", [("S1", 1), (pr2, -1), ("T", -1)], [("T", 1)]) + sq("I", [("AB", 1), ("X", -1)])
          + sq("S2", [("Z", 1), ("AB", 1), ("X", -1)]) + lin("H", [("AB", 1), ("X", -1)]))
    # E = 4I ; J = H E ; L1 = D - 2Y ; V = X E ; Z' = S2 - T - I
    a3 = (mul("J", [("H", 4)], [("I", 1)]) + mul("AV", [("X", 4)], [("I", 1)])
          + lin("L1", [("D", 1), ("Y", -2)]) + lin("ZP", [("S2", 1), ("T", -1), ("I", -1)]))
    # X' = L1^2 - J - 2V ; YJ = Y J ; T' = Z'^2 ; b = -2 L1 PX ; c = 2 Z' PY ; LA1 = 2 L1 px ; S3 = (py + Z')^2
    a4 = (sq_plus("XN", [("L1", 1)], [("J", -1), ("AV", -2)]) + mul("YJ", [("Y", 1)], [("J", 1)])
          + sq("TP", [("ZP", 1)]) + smul("LB", [("L1", -2)], "PX") + smul("LC", [("ZP", 2)], "PY")
          + mul("LA1", [("L1", 2)], [(px, 1)]) + sq("S3", [(py, 1), ("ZP", 1)]))
    # Y' = (V - X') L1 - 2 YJ ; a = LA1 - (S3 - r2 - T') ; X, Z, T <- X', Z', T'
    a5 = (mul("Y", [("AV", 1), ("XN", -1)], [("L1", 1)], extra=[("YJ", -2)])
          + lin("LA", [("LA1", 1), ("S3", -1), (pr2, 1), ("TP", 1)])
          + lin("X", [("XN", 1)]) + lin("Z", [("ZP", 1)]) + lin("T", [("TP", 1)]))
    return [a1, a2, a3, a4, a5]


# ---- homogeneous projective G2 steps (the Miller loop's point R lives in X, Y, Z
# with the Z register holding W = Z/xi, so that b' Z^2 = (3/xi) xi^2 W^2 = 3 xi W^2
# needs no multiplication by the constant b'). Textbook formulas: Costello, Lange,
# Naehrig (PKC 2010) doubling / add-1998-cmo-2 mixed addition, with the lines of
# Aranha et al. (Eurocrypt 2011) for the D-type twist; each output is a lazy sum of
# products of the previous round's values, so a doubling takes 2 rounds and an
# addition 3 (x/crypto's Jacobian lineFunctionDouble/Add take 3 and 5). The lines
# differ from x/crypto's by Fp2 factors and the points are the same points in other
# coordinates; the final exponentiation removes Fp2 factors, so the pairing (and
# every verdict) is unchanged for points of the prime-order group.
PD = {"XY": "A", "B": "B", "U": "S", "YW": "C", "X2": "G"}            # doubling temporaries
PA = {"TH": "AB", "LAM": "S1", "D": "D", "C": "I", "K": "S2", "N": "H", "J": "J", "V": "AV", "YL": "L1"}


def _xi_lc(name):
    """component lincombs of xi * name: ((3x + y), (3y - x))."""
    x, y = comp(name, "x"), comp(name, "y")
    return [(x, 3), (y, 1)], [(y, 3), (x, -1)]


def prog_double_proj(sfx=""):
    """T = (X : Y : xi W) -> 2T (scaled by 4) and the tangent line at (PX, PY):
       XY, B = Y^2, U = 9 xi W^2 (= 3 b' Z^2), YW, X2 = X^2
       X' = 2 XY (B - 3U), Y' = (B + 3U)^2 - 12 U^2, W' = 8 B YW
       line c + b w + a w^3: c = -2 xi YW PY, b = 3 X2 PX, a = U - B"""
    wx, wy = comp("Z", "x"), comp("Z", "y")
    u = [Lane(comp(PD["U"], "x"), [([(wx, 6)], [(wy, 9)]), ([(wy, 9), (wx, 9)], [(wy, 1), (wx, -1)])]),
         Lane(comp(PD["U"], "y"), [([(wy, 9), (wx, 9)], [(wy, 3), (wx, -3)]), ([(wx, -18)], [(wy, 1)])])]
    r1 = (mul(PD["XY"], [("X", 1)], [("Y", 1)]) + sq(PD["B"], [("Y", 1)]) + u
          + mul(PD["YW"], [("Y", 1)], [("Z", 1)]) + sq(PD["X2"], [("X", 1)]) + fixed_line_eval(sfx))
    b, uu = PD["B"], PD["U"]
    y3 = [Lane(comp("Y", c), sq_terms([(b, 1), (uu, 3)], c) + sq_terms([(uu, 1)], c, k=-12)) for c in "xy"]
    cx, cy = _xi_lc(PD["YW"])
    lc = [Lane(comp("LC" + sfx, "x"), [(scale(cx, -2), scal("PY"))]),
          Lane(comp("LC" + sfx, "y"), [(scale(cy, -2), scal("PY"))])]
    r2 = (mul("X", [(PD["XY"], 2)], [(b, 1), (uu, -3)]) + y3 + mul("Z", [(b, 8)], [(PD["YW"], 1)])
          + lc + smul("LB" + sfx, [(PD["X2"], 3)], "PX") + lin("LA" + sfx, [(uu, 1), (b, -1)]))
    return [r1, r2]


def prog_add_proj(px, py, sfx=""):
    """T = (X : Y : xi W) -> T + (px, py) and the line through them at (PX, PY):
       TH = Y - py xi W, LAM = X - px xi W
       D = LAM^2, C = TH^2, K = W LAM, N = X LAM, J = TH LAM, V = W TH, YL = Y LAM
       X' = D D + xi K C - 2 N D, Y' = J (3N - D) - xi V C - YL D, W' = K D
       line: c = LAM PY, b = -TH PX, a = TH px - LAM py"""
    wxi = _xi_lc("Z")

    def diff(dst, base, pt):
        # dst = base - pt * xi W
        out = []
        ptx, pty = comp(pt, "x"), comp(pt, "y")
        for c in "xy":
            if c == "x":   # (pt xi W).x = pt.x (xi W).y + pt.y (xi W).x
                slots = [([(ptx, -1)], wxi[1]), ([(pty, -1)], wxi[0])]
            else:          # (pt xi W).y = pt.y (xi W).y - pt.x (xi W).x
                slots = [([(pty, -1)], wxi[1]), ([(ptx, 1)], wxi[0])]
            out.append(Lane(comp(dst, c), slots + [([(comp(base, c), 1)], one())]))
        return out

    th, lam = PA["TH"], PA["LAM"]
    r1 = diff(th, "Y", py) + diff(lam, "X", px) + fixed_line_eval(sfx)
    r2 = (sq(PA["D"], [(lam, 1)]) + sq(PA["C"], [(th, 1)]) + mul(PA["K"], [("Z", 1)], [(lam, 1)])
          + mul(PA["N"], [("X", 1)], [(lam, 1)]) + mul(PA["J"], [(th, 1)], [(lam, 1)])
          + mul(PA["V"], [("Z", 1)], [(th, 1)]) + mul(PA["YL"], [("Y", 1)], [(lam, 1)]))
    d, cc, k, n, j, v, yl = (PA[x] for x in ("D", "C", "K", "N", "J", "V", "YL"))
    kx, ky = _xi_lc(k)
    vx, vy = _xi_lc(v)
    ccx, ccy = [(comp(cc, "x"), 1)], [(comp(cc, "y"), 1)]

    def xi_times_c(ax, ay, c, sign=1):
        # component c of sign * (ax i + ay) * C
        if c == "x":
            return [(scale(ax, sign), ccy), (scale(ay, sign), ccx)]
        return [(scale(ay, sign), ccy), (scale(neg(ax), sign), ccx)]

    x3 = [Lane(comp("X", c), sq_terms([(d, 1)], c) + xi_times_c(kx, ky, c) + prod_terms([(n, -2)], [(d, 1)], c))
          for c in "xy"]
    y3 = [Lane(comp("Y", c), prod_terms([(j, 1)], [(n, 3), (d, -1)], c) + xi_times_c(vx, vy, c, -1)
               + prod_terms([(yl, -1)], [(d, 1)], c)) for c in "xy"]
    la = [Lane(comp("LA" + sfx, c), prod_terms([(th, 1)], [(px, 1)], c) + prod_terms([(lam, -1)], [(py, 1)], c))
          for c in "xy"]
    r3 = (x3 + y3 + mul("Z", [(k, 1)], [(d, 1)]) + smul("LC" + sfx, [(lam, 1)], "PY")
          + smul("LB" + sfx, [(th, -1)], "PX") + la)
    return [r1, r2, r3]


def prog_cyc_sqr():
    """Granger-Scott squaring of f = (c0 + c3 s) + (c1 + c4 s) w + (c2 + c5 s) w^2
    (s = w^3, s^2 = xi) in the cyclotomic subgroup:
        A^2 = (a^2 + xi b^2) + ((a + b)^2 - a^2 - b^2) s = (a^2 + xi b^2) + 2ab s
        c0' = 3 (A^2)_0 - 2 c0      c3' = 3 (A^2)_1 + 2 c3        (A = (c0, c3))
        c2' = 3 (B^2)_0 - 2 c2      c5' = 3 (B^2)_1 + 2 c5        (B = (c1, c4))
        c1' = 3 xi (C^2)_1 + 2 c1   c4' = 3 (C^2)_0 - 2 c4        (C = (c2, c5))"""
    lanes = []

    def a0(a, b, c):  # component c of 3 (a^2 + xi b^2)
        bx = sq_terms([(b, 1)], "x")
        by = sq_terms([(b, 1)], "y")
        return [(scale(x, 3), y) for x, y in sq_terms([(a, 1)], c) + xi_terms(bx, by, c)]

    def a1(a, b, c, k=3):  # component c of k * 2ab
        return prod_terms([(a, 2 * k)], [(b, 1)], c)

    for c in "xy":
        lanes.append(Lane(comp("D0", c), a0("A0", "A3", c) + [(fp2_comp([("A0", -2)], c), one())]))
        lanes.append(Lane(comp("D3", c), a1("A0", "A3", c) + [(fp2_comp([("A3", 2)], c), one())]))
        lanes.append(Lane(comp("D2", c), a0("A1", "A4", c) + [(fp2_comp([("A2", -2)], c), one())]))
        lanes.append(Lane(comp("D5", c), a1("A1", "A4", c) + [(fp2_comp([("A5", 2)], c), one())]))
        lanes.append(Lane(comp("D4", c), a0("A2", "A5", c) + [(fp2_comp([("A4", -2)], c), one())]))
        # 3 xi (C^2)_1 = xi * 6 c2 c5
        px = prod_terms([("A2", 6)], [("A5", 1)], "x")
        py = prod_terms([("A2", 6)], [("A5", 1)], "y")
        lanes.append(Lane(comp("D1", c), xi_terms(px, py, c) + [(fp2_comp([("A1", 2)], c), one())]))
    return [lanes]


def prog_cyc_sqr_x():
    """Granger-Scott squaring with at most 3 products per lane (the operand
    combinations are shared by the team's pre-pass): per group (a, b),
        3(a^2 + xi b^2).x = (6ax) ay + (18bx) by + 3(by + bx)(by - bx)
        3(a^2 + xi b^2).y = 3(ay + ax)(ay - ax) - (6bx) by + 9(by + bx)(by - bx)
        6ab = (6ax by + 6ay bx) i + (6ay by - 6ax bx)
        6 xi ab = (6(3ax + ay) by + 6(3ay - ax) bx) i + (6(3ay - ax) by - 6(3ax + ay) bx)
    plus -2c (squared lanes) or +2c (product lanes) as a linear term."""
    def e(name, c):
        return comp(name, c)

    lanes = []
    groups = {0: ("A0", "A3"), 1: ("A1", "A4"), 2: ("A2", "A5")}
    # output coefficient k -> (group, kind): sq = a^2 + xi b^2 part, ab = 2ab part, xi = 2 xi ab part
    kinds = {0: (0, "sq"), 3: (0, "ab"), 2: (1, "sq"), 5: (1, "ab"), 4: (2, "sq"), 1: (2, "xi")}
    for k in range(6):
        g, kind = kinds[k]
        a, b = groups[g]
        ax, ay, bx, by = e(a, "x"), e(a, "y"), e(b, "x"), e(b, "y")
        for c in "xy":
            if kind == "sq":
                if c == "x":
                    slots = [([(ax, 6)], [(ay, 1)]), ([(bx, 18)], [(by, 1)]),
                             ([(by, 3), (bx, 3)], [(by, 1), (bx, -1)])]
                else:
                    slots = [([(ay, 3), (ax, 3)], [(ay, 1), (ax, -1)]), ([(bx, -6)], [(by, 1)]),
                             ([(by, 9), (bx, 9)], [(by, 1), (bx, -1)])]
                lin = [(e(f"A{k}", c), -2)]
            elif kind == "ab":
                if c == "x":
                    slots = [([(ax, 6)], [(by, 1)]), ([(ay, 6)], [(bx, 1)])]
                else:
                    slots = [([(ay, 6)], [(by, 1)]), ([(ax, -6)], [(bx, 1)])]
                lin = [(e(f"A{k}", c), 2)]
            else:
                u = [(ax, 18), (ay, 6)]
                v = [(ay, 18), (ax, -6)]
                if c == "x":
                    slots = [(u, [(by, 1)]), (v, [(bx, 1)])]
                else:
                    slots = [(v, [(by, 1)]), (u, [(bx, -1)])]
                lin = [(e(f"A{k}", c), 2)]
            lanes.append(Lane(comp(f"D{k}", c), slots + [(lin, one())]))
    return [lanes]


def prog_cyc_sqr_x_shared():
    """CYC_SQR_X's forms rewritten so that the lanes share their operand
    combinations (r06, the 12-lane teams: 24 pre-pass values instead of 31,
    two per lane on lanes 0..11 instead of three). The b-part of a squared
    group's two lanes,
        3(a^2 + xi b^2).x  b-part:  3 by^2 + 18 bx by - 3 bx^2 = bx V1 + by V2
        3(a^2 + xi b^2).y  b-part:  9 by^2 -  6 bx by - 9 bx^2 = by V1 + (-bx) V2
    with V1 = 9 by - 3 bx, V2 = 9 bx + 3 by, uses three values (V1, V2, -bx)
    where CYC_SQR_X uses five (18 bx, 3(by + bx), by - bx, -6 bx,
    9(by + bx)); the xi lanes of group 2 share -bx. Still at most three
    products per lane, plus -2c / +2c as a linear term."""
    def e(name, c):
        return comp(name, c)

    lanes = []
    groups = {0: ("A0", "A3"), 1: ("A1", "A4"), 2: ("A2", "A5")}
    kinds = {0: (0, "sq"), 3: (0, "ab"), 2: (1, "sq"), 5: (1, "ab"), 4: (2, "sq"), 1: (2, "xi")}
    for k in range(6):
        g, kind = kinds[k]
        a, b = groups[g]
        ax, ay, bx, by = e(a, "x"), e(a, "y"), e(b, "x"), e(b, "y")
        v1 = [(by, 9), (bx, -3)]
        v2 = [(bx, 9), (by, 3)]
        nbx = [(bx, -1)]
        for c in "xy":
            if kind == "sq":
                if c == "x":
                    slots = [([(ax, 6)], [(ay, 1)]), ([(bx, 1)], v1), ([(by, 1)], v2)]
                else:
                    slots = [([(ay, 3), (ax, 3)], [(ay, 1), (ax, -1)]), ([(by, 1)], v1), (nbx, v2)]
                lin = [(e(f"A{k}", c), -2)]
            elif kind == "ab":
                if c == "x":
                    slots = [([(ax, 6)], [(by, 1)]), ([(ay, 6)], [(bx, 1)])]
                else:
                    slots = [([(ay, 6)], [(by, 1)]), ([(ax, -6)], [(bx, 1)])]
                lin = [(e(f"A{k}", c), 2)]
            else:
                u = [(ax, 18), (ay, 6)]
                v = [(ay, 18), (ax, -6)]
                if c == "x":
                    slots = [(u, [(by, 1)]), (v, [(bx, 1)])]
                else:
                    slots = [(v, [(by, 1)]), (u, nbx)]
                lin = [(e(f"A{k}", c), 2)]
            lanes.append(Lane(comp(f"D{k}", c), slots + [(lin, one())]))
    return [lanes]


def prog_sqr12():
    """f^2 in Fp2[w]/(w^6 - xi): c_k = sum_{i<=j, i+j = k mod 6} (2 - [i==j]) a_i a_j xi^[i+j>=6]."""
    def xi_prod(i, j, c, mult):
        # component c of mult * (xi a_i) * a_j, xi a = (3x + y) i + (3y - x)
        ux = [(comp(f"A{i}", "x"), 3 * mult), (comp(f"A{i}", "y"), mult)]
        uy = [(comp(f"A{i}", "y"), 3 * mult), (comp(f"A{i}", "x"), -mult)]
        vx, vy = [(comp(f"A{j}", "x"), 1)], [(comp(f"A{j}", "y"), 1)]
        if c == "x":
            return [(ux, vy), (uy, vx)]
        return [(uy, vy), (neg(ux), vx)]

    lanes = []
    for k in range(6):
        for c in "xy":
            slots = []
            for i in range(6):
                for j in range(i, 6):
                    if (i + j) % 6 != k:
                        continue
                    mult = 1 if i == j else 2
                    if i + j >= 6:
                        slots += xi_prod(i, j, c, mult)
                    elif i == j:
                        slots += sq_terms([(f"A{i}", 1)], c)
                    else:
                        slots += prod_terms([(f"A{i}", mult)], [(f"A{j}", 1)], c)
            lanes.append(Lane(comp(f"D{k}", c), slots))
    return [lanes]


def xi_lc(lx, ly):
    """components of xi * (lx i + ly) for Fp lincombs lx, ly: (3lx + ly, 3ly - lx)."""
    return add(scale(lx, 3), ly), add(scale(ly, 3), neg(lx))


def prog_mul12():
    """dst = A * B in Fp2[w]/(w^6 - xi): lane (k, c) sums over i the component c of
    A_i' B_j, j = k - i mod 6, A_i' = xi A_i when k - i < 0 (x/crypto gfP12.Mul)."""
    lanes = []
    for k in range(6):
        for c in "xy":
            slots = []
            for i in range(6):
                j = (k - i) % 6
                ax, ay = [(comp(f"A{i}", "x"), 1)], [(comp(f"A{i}", "y"), 1)]
                if k - i < 0:
                    ax, ay = xi_lc(ax, ay)
                bx, by = [(comp(f"B{j}", "x"), 1)], [(comp(f"B{j}", "y"), 1)]
                if c == "x":
                    slots += [(ax, by), (ay, bx)]
                else:
                    slots += [(ay, by), (neg(ax), bx)]
            lanes.append(Lane(comp(f"D{k}", c), slots))
    return [lanes]


def prog_line(la, lb, lc):
    """dst = A * (lc + lb w + la w^3) (sparse line, coefficients in F registers);
    xi is applied to the line coefficient of a wrapped term."""
    lanes = []
    for k in range(6):
        for c in "xy":
            slots = []
            for jpos, L in ((0, lc), (1, lb), (3, la)):
                i = k - jpos
                lx, ly = [(comp(L, "x"), 1)], [(comp(L, "y"), 1)]
                if i < 0:
                    i += 6
                    lx, ly = xi_lc(lx, ly)
                fx, fy = [(comp(f"A{i}", "x"), 1)], [(comp(f"A{i}", "y"), 1)]
                if c == "x":
                    slots += [(fx, ly), (fy, lx)]
                else:
                    slots += [(fy, ly), (fx, neg(lx))]
            lanes.append(Lane(comp(f"D{k}", c), slots))
    return [lanes]


def prog_line_n(lb, lc):
    """dst = A * (lc + lb w + w^3): a G2Base line divided by its constant
    coefficient a (bn256_kernels.hip k_g2_lines; the Fp2 factor a is removed by
    the final exponentiation), so the w^3 part is A * w^3, a linear term (a
    coefficient shift, xi on the wrapped ones): 4 products per lane instead of
    prog_line's 6."""
    lanes = []
    for k in range(6):
        for c in "xy":
            slots = []
            for jpos, L in ((0, lc), (1, lb)):
                i = k - jpos
                lx, ly = [(comp(L, "x"), 1)], [(comp(L, "y"), 1)]
                if i < 0:
                    i += 6
                    lx, ly = xi_lc(lx, ly)
                fx, fy = [(comp(f"A{i}", "x"), 1)], [(comp(f"A{i}", "y"), 1)]
                if c == "x":
                    slots += [(fx, ly), (fy, lx)]
                else:
                    slots += [(fy, ly), (fx, neg(lx))]
            i = k - 3
            fx, fy = [(comp(f"A{i % 6}", "x"), 1)], [(comp(f"A{i % 6}", "y"), 1)]
            if i < 0:
                fx, fy = xi_lc(fx, fy)   # xi * A_{k+3}
            slots.append((fx if c == "x" else fy, one()))
            lanes.append(Lane(comp(f"D{k}", c), slots))
    return [lanes]


PROGRAMS = {
    "DBL": prog_double(),
    "ADD_POS": prog_add("QX", "QY", "R2"),
    "ADD_NEG": prog_add("QX", "NQY", "R2"),
    "ADD_F1": prog_add("P1X", "P1Y", "P1R2"),
    "ADD_F2": prog_add("P2X", "QY", "R2"),
    "CYC_SQR": prog_cyc_sqr(),
    "SQR12": prog_sqr12(),
    "MUL12": prog_mul12(),
    "LINE_PK": prog_line("LA", "LB", "LC"),
    "LINE_FIX": prog_line_n("FB", "FC"),
    "CYC_SQR_X": prog_cyc_sqr_x(),
    "PDBL": prog_double_proj(),
    "PADD_POS": prog_add_proj("QX", "QY"),
    "PADD_NEG": prog_add_proj("QX", "NQY"),
    "PADD_F1": prog_add_proj("P1X", "P1Y"),
    "PADD_F2": prog_add_proj("P2X", "QY"),
}
# The G2Base lines are normalised (a = 1): LINE_FIX = prog_line_n.
# Sig-only Miller loop (bn256_gt.hip k_verify_sig): the G2Base line at -sig is
# evaluated on lanes 12..15 beside f^2 (SDBL) or beside f * the previous line
# (LFEV), rounds whose Fp12 jobs leave those lanes idle anyway; FEVAL alone.
PROGRAMS["FEVAL"] = [fixed_line_eval()]
PROGRAMS["SDBL"] = [prog_sqr12()[0] + fixed_line_eval()]
PROGRAMS["LFEV"] = [prog_line_n("FB", "FC")[0] + fixed_line_eval()]
# Fp12 product in the compact GT-fold team layout (context FOLD below)
PROGRAMS["MUL12F"] = prog_mul12()
# k_verify_sig12 (bn256_sig12.hip): the sig-only pairing on FIVE 12-lane teams
# per wave (make_team12). The G2Base lines arrive evaluated at -sig
# (k_sig_lines), so the Miller loop is f^2 (SQR12) and f * line (LINE_FIX)
# with nothing beside them on lanes 12..15, and every pre-pass value lives on
# lanes 0..11 (PRE_LANES).
PROGRAMS["SQR12_12"] = prog_sqr12()
PROGRAMS["LINE_FIX_12"] = prog_line_n("FB", "FC")
PROGRAMS["MUL12_12"] = prog_mul12()
PROGRAMS["CYC_SQR_X_12"] = prog_cyc_sqr_x_shared()  # r06: 24 pre-pass values (two per lane)
# programs also emitted in the single-phase table format (bn256_g2sched.h)
LEGACY = ("DBL", "ADD_POS", "ADD_NEG", "ADD_F1", "ADD_F2", "CYC_SQR", "SQR12")


# ------------------------------------------------------------------ checks + interpreter
def bound(terms):
    return sum(abs(k) for _, k in terms)


def check_round(lanes, name):
    assert len(lanes) <= 16, f"{name}: {len(lanes)} lanes"
    dsts = [l.dst for l in lanes]
    assert len(set(dsts)) == len(dsts), f"{name}: duplicate destinations"
    worst = 0
    for l in lanes:
        assert len(l.slots) <= MAX_NSLOT, f"{name}: {len(l.slots)} slots"
        t = 0
        for a, b in l.slots:
            assert len(a) <= MAX_TERMS and len(b) <= MAX_TERMS, f"{name}: too many terms {a} {b}"
            # int32 limb sums in g2_lincomb: |v + K p_i| <= (pos + neg) * 2^26 < 2^31
            for terms in (a, b):
                pos = sum(k for _, k in terms if k > 0)
                negs = sum(-k for _, k in terms if k < 0)
                assert pos + negs <= 30, f"{name}: coefficient range {terms}"
            t += bound(a) * bound(b)
        # REDC output < (t / R_OVER_P + 1) p must stay below 2p (acc_reduce + csub)
        assert t / R_OVER_P + 1 < 2, f"{name}: product bound {t}"
        # 64-bit columns: limbs < 2^26 * sum|c|; 10 terms per column per slot
        worst = max(worst, t)
    return worst


def run_program(prog, F):
    """Interprets a program on an index -> residue map (plain values mod p)."""
    for lanes in prog:
        out = {}
        for l in lanes:
            acc = 0
            for a, b in l.slots:
                va = sum(k * F[r] for r, k in a)
                vb = sum(k * F[r] for r, k in b)
                acc += va * vb
            out[l.dst] = acc % P
        F.update(out)
    return F


def validate(seed=1):
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
    from oracle import bn256_oracle as O

    rng = random.Random(seed)
    for name, prog in PROGRAMS.items():
        if name not in LEGACY:
            continue
        for i, r in enumerate(prog):
            check_round(r, f"{name}[{i}]")
    for trial in range(3):
        Q = O.g2_mul(O.G2_GEN, rng.randrange(1, O.ORDER))
        Hp = O.g1_mul(O.G1_GEN, rng.randrange(1, O.ORDER))
        Rj = O.jac_mul(O.FP2_OPS, O.to_jac(O.FP2_OPS, Q), rng.randrange(2, 1000))
        r = (Rj[0], Rj[1], Rj[2], O.f2_sqr(Rj[2]))
        F = {i: rng.randrange(P) for i in list(range(NREGS)) + list(range(SLOT_A, SLOT_A + 12))
             + list(range(SLOT_B, SLOT_B + 12))}
        F[REG["ZERO"]] = 0
        F[REG["ONE"]] = 1
        F[REG["PX"]], F[REG["PY"]] = Hp

        def put(n, v):
            F[comp(n, "x")], F[comp(n, "y")] = v

        for n, v in zip(("X", "Y", "Z", "T"), r):
            put(n, v)
        put("QX", Q[0])
        put("QY", Q[1])
        put("NQY", O.f2_neg(Q[1]))
        put("R2", O.f2_sqr(Q[1]))
        a, b, c, r_new = O._line_double(r, *Hp)
        G = run_program(PROGRAMS["DBL"], dict(F))
        assert [(G[comp(n, "x")], G[comp(n, "y")]) for n in ("X", "Y", "Z", "T")] == list(r_new), "DBL point"
        assert [(G[comp(n, "x")], G[comp(n, "y")]) for n in ("LA", "LB", "LC")] == [a, b, c], "DBL line"
        for prog, pq in (("ADD_POS", (Q[0], Q[1])), ("ADD_NEG", (Q[0], O.f2_neg(Q[1])))):
            a, b, c, r_new = O._line_add(r, pq, *Hp, O.f2_sqr(pq[1]))
            G = run_program(PROGRAMS[prog], dict(F))
            assert [(G[comp(n, "x")], G[comp(n, "y")]) for n in ("X", "Y", "Z", "T")] == list(r_new), prog
            assert [(G[comp(n, "x")], G[comp(n, "y")]) for n in ("LA", "LB", "LC")] == [a, b, c], prog + " line"
        # Fp12 squarings: a random element, and a cyclotomic one
        f = [(rng.randrange(P), rng.randrange(P)) for _ in range(6)]
        cyc = O.f12_mul(O.f12_conj(f), O.f12_inv(f))
        cyc = O.f12_mul(cyc, O.f12_frob2(cyc))
        for prog, val in (("SQR12", f), ("CYC_SQR", cyc)):
            G = dict(F)
            for k in range(6):
                G[comp(f"A{k}", "x")], G[comp(f"A{k}", "y")] = val[k]
            G = run_program(PROGRAMS[prog], G)
            got = [(G[comp(f"D{k}", "x")], G[comp(f"D{k}", "y")]) for k in range(6)]
            assert got == O.f12_sqr(val), prog
    return True


# ------------------------------------------------------------------ two-phase compilation (bn256_xprog.h)
# New operand space: 0..127 F, 128..143 slot A, 144..159 slot B, 160.. scratch.
X_SLOT_B = 144
X_SCR = 160
P_LIMB_TOP = P >> 234


# Negations in a pre-pass or a linear term subtract x from a multiple of p
# re-spread limb-wise, (NEG_MULT p)'' below: every limb of it dominates the
# same limb of any element. Elements may be LAZY, below 2p instead of p: the
# cyclotomic squaring leaves its result unreduced (LAZY_PROGRAMS), so the
# multiple is 4p, whose top limb dominates the top limb of anything below 2p.
NEG_MULT = 4


def _pneg_limbs(m):
    """(m p)'': m p re-spread so limb l >= 2^26 (l < 9) and the top limb is (m p >> 234) - 1."""
    v = m * P
    q = [(v >> (26 * l)) & ((1 << 26) - 1) for l in range(9)] + [v >> 234]
    out = [q[0] + (1 << 26)] + [q[l] + (1 << 26) - 1 for l in range(1, 9)] + [q[9] - 1]
    assert sum(x << (26 * l) for l, x in enumerate(out)) == v
    return out


P2N = _pneg_limbs(NEG_MULT)                          # the negation constant (HG_P2N)
CANON_LIMB = [(1 << 26) - 1] * 9 + [P_LIMB_TOP]      # limb bounds of a canonical element
LAZY_LIMB = [(1 << 26) - 1] * 9 + [(2 * P - 1) >> 234]  # ... of an element below 2p
NEG_LIMB = list(P2N)                                 # limb bounds of (4p)'' - x
assert all(a <= b for a, b in zip(LAZY_LIMB, P2N)), "the negation constant must dominate every element"
# programs whose rounds with linear terms leave their result in [0, 2p)
# (x_round's LZ: no final conditional subtraction). Every reader of their
# output must be a team program, which takes elements below 2p: in
# t12_pow_v_x and team_final_exp (bn256_xprog.h, bn256_pairing.h) each
# squaring feeds the next squaring or a MUL12, whose result is canonical.
LAZY_PROGRAMS = ("CYC_SQR_X", "CYC_SQR_X_12")


def _xsrc(r):
    """old register code -> new operand code"""
    if r >= SLOT_B:
        return X_SLOT_B + (r - SLOT_B)
    return r


class XRound:
    """A compiled round. Each lane runs one job (prod, lin -> dst) or, in a
    fused round, a second independent job (prod2, lin2 -> dst2) after the
    first: two programs' rounds share one pre-pass, table fetch and sync."""
    def __init__(self, nv, nt, np_, nl, lanes, name, np2=0, nl2=0):
        self.nv, self.nt, self.np, self.nl, self.lanes, self.name = nv, nt, np_, nl, lanes, name
        self.np2, self.nl2 = np2, nl2
        self.ks1 = self.ks2 = 0  # Karatsuba products per job (set by check_xround)
        self.ef = 0  # the first product's operands are plain elements (compile_round)

        def negk(terms):
            return sum(-k for _, k in terms if k < 0)
        self.kp = max([negk(t) for L in lanes for d, t in L["pre"] if d != NONE] or [0])
        self.kl1 = max([negk(L["lin"]) for L in lanes] or [0])
        self.kl2 = max([negk(L.get("lin2", [])) for L in lanes] or [0])

    @property
    def fused(self):
        return self.np2 > 0 or self.nl2 > 0

    def words(self):
        nhalves = self.nv * (1 + self.nt) + 2 * self.np + self.nl + 1
        if self.fused:
            nhalves += 2 * self.np2 + self.nl2 + 1
        return (nhalves + 1) // 2

    def lane_halves(self, t):
        """16-bit entries for bound rounds (bn256_xprog.h): operands/destinations
        as byte offsets (0xffff none), terms as element << 8 | int8 coef."""
        L = self.lanes[t]
        h = []
        off = lambda e: 0xFFFF if e == NONE else 40 * e  # noqa: E731
        for dst, terms in L["pre"]:
            h.append(off(dst))
            for src, c in terms:
                assert -128 <= c <= 127
                h.append((src << 8) | (c & 255))
        for u, v in L["prod"]:
            h += [off(u), off(v)]
        for src, c in L["lin"]:
            h.append((src << 8) | (c & 255))
        h.append(off(L["dst"]))
        if self.fused:
            for u, v in L["prod2"]:
                h += [off(u), off(v)]
            for src, c in L["lin2"]:
                h.append((src << 8) | (c & 255))
            h.append(off(L["dst2"]))
        h += [0] * (2 * self.words() - len(h))
        return h

    def lane_bytes(self, t):
        L = self.lanes[t]
        b = []
        for dst, terms in L["pre"]:
            b.append(dst)
            for src, c in terms:
                b += [src, c & 255]
        for u, v in L["prod"]:
            b += [u, v]
        for src, c in L["lin"]:
            b += [src, c & 255]
        b.append(L["dst"])
        b += [0] * (4 * self.words() - len(b))
        return b


def compile_round(lanes, name, scratch_cap, lanes2=None, pre_lanes=16):
    """pre_lanes: lanes that evaluate the pre-pass values (16, or 12 for
    programs that also run in 12-lane teams: PRE_LANES)."""
    one_lc = [(REG["ONE"], 1)]
    values = {}      # canonical lincomb -> scratch code
    order = []

    def operand(lc):
        lc = [(r, k) for r, k in lc if k != 0] or [(REG["ZERO"], 1)]
        if len(lc) == 1 and lc[0][1] == 1:
            return _xsrc(lc[0][0])
        key = tuple(sorted((_xsrc(r), k) for r, k in lc))
        if key not in values:
            values[key] = X_SCR + len(order)
            order.append(key)
        return values[key]

    def jobs(ls):
        per = []
        for l in ls:
            prods, lins = [], []
            for a, b in l.slots:
                if list(b) == one_lc:
                    lins += [(_xsrc(r), k) for r, k in a if k != 0]
                elif list(a) == one_lc:
                    lins += [(_xsrc(r), k) for r, k in b if k != 0]
                else:
                    prods.append((operand(a), operand(b)))
            per.append((l.dst, prods, lins))
        assert len(per) <= 16, name
        return per

    per_lane = jobs(lanes)
    per_lane2 = jobs(lanes2) if lanes2 is not None else []
    # early first product (x_round's EF): when every lane has a product whose
    # operands are both plain elements (no pre-pass value), it goes first and
    # its operands are read together with the pre-pass's inputs, so the
    # products start without waiting for a second LDS round trip
    ef = int(lanes2 is None and any(p for _, p, _ in per_lane)
             and all(any(u < X_SCR and v < X_SCR for u, v in p) for _, p, _ in per_lane if p))
    if ef:
        for i, (d, p, q) in enumerate(per_lane):
            if p:
                k = next(j for j, (u, v) in enumerate(p) if u < X_SCR and v < X_SCR)
                per_lane[i] = (d, [p[k]] + p[:k] + p[k + 1:], q)
    if lanes2 is not None:
        # the first job's destinations are written after the second job reads: no overlap
        d1 = {d for d, _, _ in per_lane}
        for _, p2, l2 in per_lane2:
            assert not ({u for u, v in p2} | {v for u, v in p2} | {s for s, _ in l2}) & d1, name
    nvals = len(order)
    assert nvals <= scratch_cap, f"{name}: {nvals} pre-pass values > scratch {scratch_cap}"
    nv = (nvals + pre_lanes - 1) // pre_lanes
    nt = max([len(k) for k in order] or [0])
    np_ = max(len(p) for _, p, _ in per_lane)
    nl = max(len(q) for _, _, q in per_lane)
    np2 = max([len(p) for _, p, _ in per_lane2] or [0])
    nl2 = max([len(q) for _, _, q in per_lane2] or [0])
    if lanes2 is not None and np2 == 0 and nl2 == 0:
        nl2 = 1  # keep the fused layout
    zero = REG["ZERO"]
    out = []
    for t in range(16):
        pre = []
        for v in range(nv):
            vi = t + pre_lanes * v
            if t < pre_lanes and vi < nvals:
                terms = list(order[vi]) + [(zero, 0)] * (nt - len(order[vi]))
                pre.append((X_SCR + vi, terms))
            else:
                pre.append((NONE, [(zero, 0)] * nt))
        dst, prods, lins = per_lane[t] if t < len(per_lane) else (NONE, [], [])
        prods = prods + [(zero, zero)] * (np_ - len(prods))
        lins = lins + [(zero, 0)] * (nl - len(lins))
        L = {"pre": pre, "prod": prods, "lin": lins, "dst": dst}
        if lanes2 is not None:
            dst2, prods2, lins2 = per_lane2[t] if t < len(per_lane2) else (NONE, [], [])
            L["prod2"] = prods2 + [(zero, zero)] * (np2 - len(prods2))
            L["lin2"] = lins2 + [(zero, 0)] * (nl2 - len(lins2))
            L["dst2"] = dst2
        out.append(L)
    xr = XRound(nv, nt, np_, nl, out, name, np2, nl2)
    xr.ef = ef
    try:
        check_xround(xr, order)
    except AssertionError:
        # the round-uniform correction overflows a bound: per-lane corrections
        xr.kp = xr.kl1 = xr.kl2 = -1
        check_xround(xr, order)
    return xr


def check_xround(xr, order):
    """Limb sums < 2^32, 64-bit columns < 2^64, REDC input < 800 p^2."""
    def src_bound(code):
        if code >= X_SCR:
            return vbound[code]
        return (2 * P, LAZY_LIMB)  # any element may be lazy (< 2p)

    # Every value of the pre-pass (and every lane's linear terms of a job) adds the
    # round-uniform correction K (2p)'' with K = the largest sum of negative
    # coefficients (xr.kp / kl1 / kl2): a compile-time constant in the executor.
    vbound = {}
    for i, key in enumerate(order):
        kp = xr.kp if xr.kp >= 0 else sum(-k for _, k in key if k < 0)  # -1: per-lane correction
        val, limbs = kp * NEG_MULT * P, [kp * x for x in P2N]
        for src, k in key:
            if k > 0:
                v, lb = src_bound(src)
                val += k * v
                limbs = [a + k * b for a, b in zip(limbs, lb)]
        assert max(limbs) < 1 << 32, f"{xr.name}: pre-pass limb overflow {key}"
        vbound[X_SCR + i] = (val, limbs)
    jobs = [(L["prod"], L["lin"], xr.kl1, xr.nl) for L in xr.lanes]
    if xr.fused:
        jobs += [(L["prod2"], L["lin2"], xr.kl2, xr.nl2) for L in xr.lanes]
    # Karatsuba per job (bn256_xprog.h x_products_ks): worth it from
    # KARATSUBA_MIN products, valid while the 5-limb half sums stay 32-bit
    def ks_ok(prods):
        return len(prods) >= KARATSUBA_MIN and all(
            max(lb[i] + lb[i + 5] for i in range(5)) < 1 << 32
            for u, v in prods for lb in (src_bound(u)[1], src_bound(v)[1]))
    xr.ks1 = int(all(ks_ok(L["prod"]) for L in xr.lanes))
    xr.ks2 = int(xr.fused and all(ks_ok(L["prod2"]) for L in xr.lanes))
    for prod, lin, kl, nl in jobs:
        L = {"prod": prod, "lin": lin}
        if kl < 0:
            kl = sum(-k for _, k in lin if k < 0)
        T, cols = 0, [0] * 21
        for u, v in L["prod"]:
            (bu, lu), (bv, lv) = src_bound(u), src_bound(v)
            T += bu * bv
            for i in range(10):
                for j in range(10):
                    cols[i + j] += lu[i] * lv[j]
        if nl > 0:
            T += kl * NEG_MULT * P * (1 << R_BITS)
            for i in range(10):
                cols[R_BITS // 26 + i] += kl * P2N[i]
        for src, k in L["lin"]:
            if k <= 0:
                continue
            b, lb = src_bound(src)
            T += k * b * (1 << R_BITS)
            for i in range(10):
                cols[R_BITS // 26 + i] += k * lb[i]
        # REDC adds up to 10 digit products (< 2^52 each) and a carry to every column
        assert max(cols) + 11 * (1 << 52) < 1 << 64, f"{xr.name}: column overflow"
        # REDC(T) < T/R + p with R = 2^286. Product-only rounds: T < p R gives a result
        # < 2p (acc_reduce, one conditional subtraction). Rounds with linear terms
        # (passed through REDC unchanged): result < T/R + p must stay below 31p, the
        # exact range of fp_reduce8 (q <= 30 keeps q * p_l inside int32).
        if nl > 0:
            assert T / (1 << R_BITS) + P < 30 * P, f"{xr.name}: REDC result {T / (1 << R_BITS) / P:.1f} p"
        else:
            assert T < P * (1 << R_BITS), f"{xr.name}: REDC input {T / P / P:.1f} p^2"


def run_xround(xr, F, A, B):
    """Interprets a compiled round on plain residues; returns {dst: value}."""
    S = {}

    def get(code):
        if code >= X_SCR:
            return S[code]
        if code >= X_SLOT_B:
            return B[code - X_SLOT_B]
        if code >= SLOT_A:
            return A[code - SLOT_A]
        return F[code]

    for L in xr.lanes:
        for dst, terms in L["pre"]:
            if dst != NONE:
                S[dst] = sum(k * get(src) for src, k in terms) % P
    out = {}
    for L in xr.lanes:
        for pk, lk, dk in (("prod", "lin", "dst"), ("prod2", "lin2", "dst2")):
            if dk not in L or L[dk] == NONE:
                continue
            acc = sum(get(u) * get(v) for u, v in L[pk]) + sum(k * get(src) for src, k in L[lk])
            assert L[dk] not in out, "two jobs write one destination"
            out[L[dk]] = acc % P
    return out


X_FETCH_WORDS = 16  # words per lane one table prefetch brings in (>= the widest round)
# programs whose pre-pass values live on lanes 0..11 only, so that they also
# run in 12-lane teams (five per wave: k_gt_chunks, make_team12)
PRE_LANES = {"MUL12F": 12, "SQR12_12": 12, "LINE_FIX_12": 12, "MUL12_12": 12, "CYC_SQR_X_12": 12}
KARATSUBA_MIN = 4   # jobs of this many products use Karatsuba (when check_xround allows)
# FE: the register file from register 2 on; ML: slots C..J during the Miller loop
# FOLD: the GT fold kernels' compact team region (bn256_gt.hip): slots F, A, B,
# then registers ZERO and ONE, then the pre-pass scratch
SCRATCH_CAP = {"FE": 48, "ML": 96, "FOLD": 48}
X_PROGRAMS = {  # name -> (program, scratch context)
    "PDBL": "ML", "PADD_POS": "ML", "PADD_NEG": "ML", "PADD_F1": "ML", "PADD_F2": "ML",
    "MDBL_1": "ML", "MDBL_2": "ML", "PDBL_1": "ML",
    "PADD_POS_1": "ML", "MADD_POS_2": "ML", "PADD_POS_3": "ML", "PADD_NEG_1": "ML", "MADD_NEG_2": "ML",
    "PADD_NEG_3": "ML", "PADD_F1_1": "ML", "MADD_F1_2": "ML", "PADD_F1_3": "ML", "PADD_F2_1": "ML",
    "MADD_F2_2": "ML", "PADD_F2_3": "ML",
    "SQR12": "ML", "LINE_PK": "ML", "LINE_FIX": "ML", "CYC_SQR": "FE", "MUL12": "FE", "CYC_SQR_X": "FE",
    "FEVAL": "ML", "SDBL": "ML", "LFEV": "ML", "MUL12F": "FOLD",
    "SQR12_12": "ML", "LINE_FIX_12": "ML", "MUL12_12": "FE", "CYC_SQR_X_12": "FE",
}


# Miller-loop programs whose rounds fuse two independent rounds (see XRound):
# name -> list of rounds, each (program, round) or ((program, round), (program, round)).
FUSED = {
    "MDBL_1": [(("SQR12", 0), ("PDBL", 0))],          # f^2 beside the doubling's first round
    "MDBL_2": [(("LINE_FIX", 0), ("PDBL", 1))],       # f * G2Base line beside its second round
    "PDBL_1": [("PDBL", 0)],                          # first iteration (f = 1: no squaring)
}
for _v in ("POS", "NEG", "F1", "F2"):
    FUSED[f"PADD_{_v}_1"] = [(f"PADD_{_v}", 0)]
    FUSED[f"MADD_{_v}_2"] = [(("LINE_FIX", 0), (f"PADD_{_v}", 1))]
    FUSED[f"PADD_{_v}_3"] = [(f"PADD_{_v}", 2)]


def _compile_fused(name, ctx):
    out = []
    for i, spec in enumerate(FUSED[name]):
        if isinstance(spec[0], tuple):
            (p1, r1), (p2, r2) = spec
            out.append(compile_round(PROGRAMS[p1][r1], f"{name}[{i}]", SCRATCH_CAP[ctx], PROGRAMS[p2][r2]))
        else:
            p1, r1 = spec
            out.append(compile_round(PROGRAMS[p1][r1], f"{name}[{i}]", SCRATCH_CAP[ctx]))
    return out


def compile_all():
    X = {}
    for name, ctx in X_PROGRAMS.items():
        if name in FUSED:
            X[name] = _compile_fused(name, ctx)
        else:
            X[name] = [compile_round(r, f"{name}[{i}]", SCRATCH_CAP[ctx], pre_lanes=PRE_LANES.get(name, 16))
                       for i, r in enumerate(PROGRAMS[name])]
    return X


def run_xprogram(rounds, F, A=None, B=None):
    """F: register dict (mutated), A/B: slot element lists; returns the D slot (dict e -> v)."""
    A = A or [0] * 12
    B = B or [0] * 12
    D = {}
    for xr in rounds:
        out = run_xround(xr, F, A, B)
        for dst, v in out.items():
            if dst < 128:
                F[dst] = v
            else:
                D[dst - 128] = v
    return D


def validate_x(seed=2):
    """The compiled programs against the oracle (same cases as validate())."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
    from oracle import bn256_oracle as O

    X = compile_all()
    rng = random.Random(seed)
    for trial in range(3):
        Q = O.g2_mul(O.G2_GEN, rng.randrange(1, O.ORDER))
        Hp = O.g1_mul(O.G1_GEN, rng.randrange(1, O.ORDER))
        Rj = O.jac_mul(O.FP2_OPS, O.to_jac(O.FP2_OPS, Q), rng.randrange(2, 1000))
        r = (Rj[0], Rj[1], Rj[2], O.f2_sqr(Rj[2]))
        F = {i: rng.randrange(P) for i in range(NREGS)}
        F[REG["ZERO"]] = 0
        F[REG["ONE"]] = 1
        F[REG["PX"]], F[REG["PY"]] = Hp

        def put(G, n, v):
            G[comp(n, "x")], G[comp(n, "y")] = v

        def getf(G, n):
            return (G[comp(n, "x")], G[comp(n, "y")])

        for n, v in zip(("X", "Y", "Z", "T"), r):
            put(F, n, v)
        put(F, "QX", Q[0])
        put(F, "QY", Q[1])
        put(F, "NQY", O.f2_neg(Q[1]))
        put(F, "R2", O.f2_sqr(Q[1]))
        # projective steps: R as (x Z : y Z : Z) with Z = xi W for a random W
        xi = (1, 3)
        aff = lambda j: (O.f2_mul(j[0], O.f2_inv(O.f2_sqr(j[2]))),  # noqa: E731
                         O.f2_mul(j[1], O.f2_inv(O.f2_mul(O.f2_sqr(j[2]), j[2]))))
        rx, ry = aff(Rj)
        Wr = (rng.randrange(1, P), rng.randrange(P))
        Zr = O.f2_mul(xi, Wr)
        put(F, "X", O.f2_mul(rx, Zr))
        put(F, "Y", O.f2_mul(ry, Zr))
        put(F, "Z", Wr)
        put(F, "P1X", O.f2_mul(Q[0], (rng.randrange(P), rng.randrange(P))))  # any affine point works
        put(F, "P1Y", (rng.randrange(P), rng.randrange(P)))

        def check_proj(G, want_r, want_line, name):
            zi = O.f2_inv(O.f2_mul(xi, getf(G, "Z")))
            got = (O.f2_mul(getf(G, "X"), zi), O.f2_mul(getf(G, "Y"), zi))
            assert got == aff(want_r), name + " point"
            la, lb, lc = (getf(G, n) for n in ("LA", "LB", "LC"))
            a, b, c = want_line
            mu = O.f2_mul(la, O.f2_inv(a))   # the lines agree up to an Fp2 factor
            assert mu != (0, 0) and (la, lb, lc) == tuple(O.f2_mul(mu, v) for v in (a, b, c)), name + " line"

        a, b, c, r_new = O._line_double(r, *Hp)
        G = dict(F)
        run_xprogram(X["PDBL"], G)
        check_proj(G, r_new, (a, b, c), "xPDBL")
        # fused Miller-loop programs: f^2 and the G2Base line beside the G2 step rounds
        f0 = [(rng.randrange(P), rng.randrange(P)) for _ in range(6)]
        flat0 = [z for pair in f0 for z in pair]
        # a normalised G2Base line (a = 1, k_g2_lines): c + b w + w^3
        fl_bx, fl_cy = (rng.randrange(P), rng.randrange(P)), (rng.randrange(P), rng.randrange(P))
        F[REG["SX"]], F[REG["NSY"]] = rng.randrange(P), rng.randrange(P)
        put(F, "FBX", fl_bx)
        put(F, "FCY", fl_cy)
        fix = (O.F2_ONE, O.f2_mul(fl_bx, (0, F[REG["SX"]])), O.f2_mul(fl_cy, (0, F[REG["NSY"]])))
        unfl = lambda D: [(D[2 * k], D[2 * k + 1]) for k in range(6)]  # noqa: E731
        G = dict(F)
        sq = run_xprogram(X["MDBL_1"], G, flat0)
        assert unfl(sq) == O.f12_sqr(f0), "xMDBL_1 square"
        d2 = run_xprogram(X["MDBL_2"], G, [sq[e] for e in range(12)])
        assert unfl(d2) == O._mul_line(O.f12_sqr(f0), *fix), "xMDBL_2 fixed line"
        check_proj(G, r_new, (a, b, c), "xMDBL")
        G = dict(F)
        run_xprogram(X["PDBL_1"], G)
        d2 = run_xprogram(X["MDBL_2"], G, flat0)
        assert unfl(d2) == O._mul_line(f0, *fix), "xPDBL_1/MDBL_2 fixed line"
        check_proj(G, r_new, (a, b, c), "xPDBL_1")
        for prog, pq in (("PADD_POS", (Q[0], Q[1])), ("PADD_NEG", (Q[0], O.f2_neg(Q[1]))),
                         ("PADD_F1", (getf(F, "P1X"), getf(F, "P1Y")))):
            a, b, c, r_new = O._line_add(r, pq, *Hp, O.f2_sqr(pq[1]))
            G = dict(F)
            run_xprogram(X[prog], G)
            check_proj(G, r_new, (a, b, c), "x" + prog)
            v = prog[5:]
            G = dict(F)
            run_xprogram(X[f"PADD_{v}_1"], G)
            d2 = run_xprogram(X[f"MADD_{v}_2"], G, flat0)
            run_xprogram(X[f"PADD_{v}_3"], G)
            assert unfl(d2) == O._mul_line(f0, *fix), "xMADD fixed line"
            check_proj(G, r_new, (a, b, c), "x" + prog + " split")
        # sig-only Miller rounds: f^2 / f * line with the next line's evaluation beside
        G = dict(F)
        sq = run_xprogram(X["SDBL"], G, flat0)
        assert unfl(sq) == O.f12_sqr(f0), "xSDBL square"
        assert (getf(G, "FB"), getf(G, "FC")) == fix[1:], "xSDBL line evaluation"
        G = dict(F)
        put(G, "FB", fix[1])
        put(G, "FC", fix[2])
        nbx, ncy = (rng.randrange(P), rng.randrange(P)), (rng.randrange(P), rng.randrange(P))
        put(G, "FBX", nbx)
        put(G, "FCY", ncy)
        d2 = run_xprogram(X["LFEV"], G, flat0)
        assert unfl(d2) == O._mul_line(f0, *fix), "xLFEV line"
        assert (getf(G, "FB"), getf(G, "FC")) == (O.f2_mul(nbx, (0, F[REG["SX"]])),
                                                  O.f2_mul(ncy, (0, F[REG["NSY"]]))), "xLFEV evaluation"
        G = dict(F)
        run_xprogram(X["FEVAL"], G)
        assert (getf(G, "FB"), getf(G, "FC")) == fix[1:], "xFEVAL"
        f = [(rng.randrange(P), rng.randrange(P)) for _ in range(6)]
        g = [(rng.randrange(P), rng.randrange(P)) for _ in range(6)]
        flat = lambda v: [z for pair in v for z in pair]  # noqa: E731
        unflat = lambda D: [(D[2 * k], D[2 * k + 1]) for k in range(6)]  # noqa: E731
        cyc = O.f12_mul(O.f12_conj(f), O.f12_inv(f))
        cyc = O.f12_mul(cyc, O.f12_frob2(cyc))
        assert unflat(run_xprogram(X["SQR12"], dict(F), flat(f))) == O.f12_sqr(f), "xSQR12"
        assert unflat(run_xprogram(X["CYC_SQR"], dict(F), flat(cyc))) == O.f12_sqr(cyc), "xCYC_SQR"
        assert unflat(run_xprogram(X["CYC_SQR_X"], dict(F), flat(cyc))) == O.f12_sqr(cyc), "xCYC_SQR_X"
        assert unflat(run_xprogram(X["MUL12"], dict(F), flat(f), flat(g))) == O.f12_mul(f, g), "xMUL12"
        assert unflat(run_xprogram(X["MUL12F"], dict(F), flat(f), flat(g))) == O.f12_mul(f, g), "xMUL12F"
        # the 12-lane (pre-pass on lanes 0..11) forms of k_verify_sig12
        assert unflat(run_xprogram(X["SQR12_12"], dict(F), flat(f))) == O.f12_sqr(f), "xSQR12_12"
        assert unflat(run_xprogram(X["CYC_SQR_X_12"], dict(F), flat(cyc))) == O.f12_sqr(cyc), "xCYC_SQR_X_12"
        assert unflat(run_xprogram(X["MUL12_12"], dict(F), flat(f), flat(g))) == O.f12_mul(f, g), "xMUL12_12"
        for name in ("SQR12_12", "LINE_FIX_12", "MUL12_12", "CYC_SQR_X_12"):
            for xr in X[name]:  # no pre-pass value on lanes 12..15
                assert all(d == NONE for L in xr.lanes[12:] for d, _ in L["pre"]), name
        G = dict(F)
        la, lb, lc = [(rng.randrange(P), rng.randrange(P)) for _ in range(3)]
        put(G, "LA", la)
        put(G, "LB", lb)
        put(G, "LC", lc)
        assert unflat(run_xprogram(X["LINE_PK"], G, flat(f))) == O._mul_line(f, la, lb, lc), "xLINE_PK"
        put(G, "FB", lb)
        put(G, "FC", lc)
        assert unflat(run_xprogram(X["LINE_FIX"], G, flat(f))) == O._mul_line(f, O.F2_ONE, lb, lc), "xLINE_FIX"
        assert unflat(run_xprogram(X["LINE_FIX_12"], G, flat(f))) == O._mul_line(f, O.F2_ONE, lb, lc), \
            "xLINE_FIX_12"
    return X


# ------------------------------------------------------------------ per-call-site instances
# Team LDS (bn256_pairing.h): 12 Fp12 slots of 12 elements, then the register
# file F; operands become absolute team element indices (slot s element e ->
# 12 s + e, register r -> 144 + r), so the executor needs no address selects.
SLOTS = ["F", "A", "B", "C", "D", "E", "G", "H", "I", "J", "K", "L"]   # enum S_F.. (bn256_pairing.h)
F_BASE = 12 * len(SLOTS)
# register base per context: FOLD keeps only ZERO and ONE, right after slot B
FOLD_F_BASE = 12 * (SLOTS.index("B") + 1)
F_BASE_CTX = {"FE": F_BASE, "ML": F_BASE, "FOLD": FOLD_F_BASE}
SCR_BASE = {"FE": F_BASE + 2, "ML": 12 * SLOTS.index("C"), "FOLD": FOLD_F_BASE + 2}
REGION_END = {"FE": F_BASE + NREGS_RUNTIME, "ML": F_BASE + NREGS_RUNTIME,
              "FOLD": FOLD_F_BASE + 2 + SCRATCH_CAP["FOLD"]}
assert SCR_BASE["FE"] + SCRATCH_CAP["FE"] <= F_BASE + NREGS_RUNTIME


def _pow_u_mul_instances(dst, sa):
    """t12_pow_u_x<dst, sa> (bn256_xprog.h): three exponentiations by v,
    a -> dst, dst -> J, J -> dst, each with the conjugate of its base in K."""
    out = []
    for d, base in ((dst, sa), ("J", dst), (dst, "J")):
        out += [("CYC_SQR_X", (d, base)), ("CYC_SQR_X", (d, d)), ("MUL12", (d, d, "K")), ("MUL12", (d, d, base))]
    return out


INSTANCES = sorted(set(
    [("MUL12", b) for b in [("F", "B", "A"), ("F", "F", "A"), ("A", "A", "B"), ("H", "C", "H"), ("I", "E", "I"),
                            ("K", "K", "H"), ("K", "K", "D"), ("J", "G", "D"), ("J", "J", "K"), ("K", "K", "C"),
                            ("K", "J", "L"), ("J", "J", "A"), ("F", "K", "J"), ("L", "F", "K"), ("A", "K", "L"),
                            ("F", "A", "B"), ("L", "A", "K"), ("F", "K", "L")]]
    # team_final_exp's exp-by-v chain (slots I <-> J, conjugate in K) and the a^u probe
    + [("CYC_SQR_X", b) for b in [("J", "I"), ("J", "J"), ("I", "J"), ("I", "I")]]
    + [("MUL12", b) for b in [("J", "J", "K"), ("J", "J", "I"), ("I", "I", "K"), ("I", "I", "J")]]
    + _pow_u_mul_instances("F", "A")
    + [("CYC_SQR_X", b) for b in [("K", "I"), ("J", "J"), ("K", "K"), ("F", "A")]]
    + [("SQR12", ("F", "F")), ("SQR12", ("F", "A")), ("LINE_PK", ("F", "F")), ("LINE_FIX", ("F", "F"))]
    # tools/opcycles.hip
    + [("CYC_SQR_X", ("A", "A")), ("SQR12", ("A", "A")), ("LINE_PK", ("A", "A"))]
    + [(g, ()) for g in ("PDBL", "PADD_POS", "PADD_NEG", "PADD_F1", "PADD_F2", "PDBL_1")]
    + [(f"PADD_{v}_{i}", ()) for v in ("POS", "NEG", "F1", "F2") for i in (1, 3)]
    + [(f"MADD_{v}_2", ("F", "F")) for v in ("POS", "NEG", "F1", "F2")]
    + [("MDBL_1", ("F", "F")), ("MDBL_2", ("F", "F"))]
    # team_final_exp_fc (bn256_pairing.h): the Fuentes-Castaneda hard part
    + [("CYC_SQR_X", ("B", "A")), ("CYC_SQR", ("I", "C"))]
    + [("MUL12", b) for b in [("B", "A", "B"), ("B", "C", "D"), ("E", "B", "J"), ("D", "A", "E"), ("A", "C", "E"),
                              ("A", "F", "A"), ("A", "G", "A"), ("G", "G", "D"), ("F", "G", "A")]]
    # bn256_gt.hip: the GT fold
    + [("MUL12F", ("A", "A", "B"))]))

# k_verify_sig's compact team region (layout "S", bn256_gt.hip): slots F, A, B,
# C, D, E, G — the sig-only Miller loop and the Fuentes-Castaneda final
# exponentiation (team_final_exp_fc_s) need no more — then the register file.
# The Miller loop's pre-pass scratch lies in slots A.. (only F is live there),
# the final exponentiation's past register ONE (the Miller registers are dead
# there), as in the full layout. 118 elements per team instead of 180: 18.9 KB
# of LDS per 4-team wave, so two pairing waves fit on a SIMD and the CU keeps
# room for a fold workgroup beside its eight pairing waves.
SIG_SLOTS = SLOTS[:7]
SIG_F_BASE = 12 * len(SIG_SLOTS)
SIG_SCR_BASE = {"FE": SIG_F_BASE + 2, "ML": 12 * SLOTS.index("A")}
SIG_INSTANCES = sorted(set(
    [("SDBL", ("F", "F")), ("LFEV", ("F", "F")), ("FEVAL", ()), ("LINE_FIX", ("F", "F"))]
    # the easy part (inversion scratch D, E) and the exponentiations by v
    # (D <-> E, conjugate of the base in G)
    + [("MUL12", b) for b in [("E", "F", "D"), ("A", "D", "E"), ("F", "B", "A"), ("F", "F", "A"),
                              ("E", "E", "G"), ("E", "E", "D"), ("D", "D", "G"), ("D", "D", "E"),
                              ("B", "A", "B"), ("B", "C", "G"), ("G", "B", "E"), ("B", "A", "G"),
                              ("A", "C", "G"), ("A", "F", "A"), ("A", "D", "A"), ("D", "D", "B"), ("F", "D", "A")]]
    + [("CYC_SQR_X", b) for b in [("E", "D"), ("E", "E"), ("D", "E"), ("D", "D"), ("A", "A"), ("B", "A")]]
    # t3 = t2^2 as a product (canonical, 21 scratch elements: the canonical
    # CYC_SQR's 34 would set the region's end)
    + [("MUL12", ("D", "C", "C"))]))
# k_verify_sig12's team region (layout "T", bn256_sig12.hip): FIVE Fp12 slots
# F, A, B, C, D — the final exponentiation parks two values (res and t0) in
# HBM while the exponentiations by u run (bn256_sigfe.h team_final_exp_fc_t),
# so five slots are live at most — then the register file (ZERO, ONE; the
# Miller loop's FB, FC; the final exponentiation's pre-pass scratch from
# register 2 on). 92 elements (94 before the r06 shared-operand squaring):
# five 12-lane teams take 18.4 KB of LDS per
# wave, so a CU holds eight pairing waves (two per SIMD) and a fold workgroup.
SIG_T_SLOTS = SLOTS[:5]
SIG_T_F_BASE = 12 * len(SIG_T_SLOTS)
SIG_T_SCR_BASE = {"FE": SIG_T_F_BASE + 2, "ML": 12 * SLOTS.index("A")}
SIG_T_INSTANCES = sorted(set(
    [("SQR12_12", ("F", "F")), ("LINE_FIX_12", ("F", "F"))]
    # the easy part and the three phases' exponentiations by v (C <-> D, the
    # conjugate of the base in B / F) and their tails
    + [("MUL12_12", b) for b in [("B", "F", "D"), ("A", "D", "B"), ("F", "B", "A"), ("F", "F", "A"),
                                 ("C", "C", "B"), ("C", "C", "F"), ("D", "D", "B"), ("D", "D", "F"),
                                 ("B", "A", "B"), ("B", "A", "F"), ("D", "A", "A"), ("D", "B", "C"),
                                 ("F", "A", "D"), ("F", "A", "F"), ("F", "C", "F"), ("D", "D", "C"), ("C", "C", "D")]]
    + [("CYC_SQR_X_12", b) for b in [("C", "F"), ("C", "C"), ("D", "C"), ("D", "D"), ("C", "D"), ("C", "B"),
                                     ("A", "A"), ("B", "A")]]))
# k_verify_ml's team region (layout "V", bn256_verify.hip, r06): the
# two-pairing Miller loop of config 2 alone — f in slot F, the pre-pass values
# of its programs right after it (MDBL_1's 50 at most), then the whole runtime
# register file — 128 elements, so a 4-team wave takes 20480 bytes of LDS and
# a CU's 160 KiB holds eight, two per SIMD (k_verify's 212-element region:
# four). The final
# exponentiation runs on the 12-lane split kernels (bn256_sig12.hip).
V_SCRATCH = 50
V_F_BASE = 12 + V_SCRATCH
V_INSTANCES = ([("MDBL_1", ("F", "F")), ("MDBL_2", ("F", "F")), ("PDBL_1", ()), ("LINE_PK", ("F", "F"))]
               + [(f"PADD_{v}_{i}", ()) for v in ("POS", "NEG", "F1", "F2") for i in (1, 3)]
               + [(f"MADD_{v}_2", ("F", "F")) for v in ("POS", "NEG", "F1", "F2")])
ALL_INSTANCES = ([(n, b, "") for n, b in INSTANCES] + [(n, b, "S") for n, b in SIG_INSTANCES]
                 + [(n, b, "T") for n, b in SIG_T_INSTANCES] + [(n, b, "V") for n, b in V_INSTANCES])




def bind(xr, binding, ctx, layout=""):
    """Translates a compiled round to absolute team element indices."""
    D, A, B = (list(binding) + [None, None, None])[:3]
    if len(binding) == 2:
        D, A = binding
        B = A
    sbase = SCR_BASE[ctx]
    fbase = F_BASE_CTX[ctx]
    region_end = REGION_END[ctx]
    if layout == "S":
        assert ctx in SIG_SCR_BASE and all(b in SIG_SLOTS for b in binding), "layout S: slots F..G only"
        sbase, fbase, region_end = SIG_SCR_BASE[ctx], SIG_F_BASE, SIG_F_BASE + NREGS_RUNTIME
    if layout == "T":
        assert ctx in SIG_T_SCR_BASE and all(b in SIG_T_SLOTS for b in binding), "layout T: slots F..D only"
        sbase, fbase, region_end = SIG_T_SCR_BASE[ctx], SIG_T_F_BASE, SIG_T_F_BASE + NREGS_RUNTIME
    if layout == "V":
        assert ctx == "ML" and all(b == "F" for b in binding), "layout V: the Miller loop on slot F"
        sbase, fbase, region_end = 12, V_F_BASE, V_F_BASE + NREGS_RUNTIME

    def src(code):
        if code >= X_SCR:
            return sbase + (code - X_SCR)
        if code >= X_SLOT_B:
            return 12 * SLOTS.index(B) + (code - X_SLOT_B)
        if code >= SLOT_A:
            return 12 * SLOTS.index(A) + (code - SLOT_A)
        assert ctx != "FOLD" or code in (REG["ZERO"], REG["ONE"]), "FOLD keeps only ZERO and ONE"
        return fbase + code

    def dst(code):
        if code == NONE:
            return NONE
        if code >= SLOT_A:
            return 12 * SLOTS.index(D) + (code - SLOT_A)
        assert ctx != "FOLD", "FOLD programs write slots only"
        return fbase + code

    lanes = []
    for L in xr.lanes:
        b = {"pre": [(NONE if d == NONE else src(d), [(src(s), c) for s, c in t]) for d, t in L["pre"]],
             "prod": [(src(u), src(v)) for u, v in L["prod"]],
             "lin": [(src(s), c) for s, c in L["lin"]], "dst": dst(L["dst"])}
        if xr.fused:
            b["prod2"] = [(src(u), src(v)) for u, v in L["prod2"]]
            b["lin2"] = [(src(s), c) for s, c in L["lin2"]]
            b["dst2"] = dst(L["dst2"])
        lanes.append(b)
    for L in lanes:
        srcs = [u for u, v in L["prod"] + L.get("prod2", [])] + [v for u, v in L["prod"] + L.get("prod2", [])]
        srcs += [s_ for s_, _ in L["lin"] + L.get("lin2", [])] + [s_ for _, t in L["pre"] for s_, _ in t]
        for v in [L["dst"], L.get("dst2", NONE)] + [d for d, _ in L["pre"]] + srcs:
            assert v == NONE or v < region_end, "index out of the kernels' team region"
        if layout == "S" and ctx == "ML":  # the Miller scratch stays inside slots A..G
            assert all(d == NONE or 12 <= d < SIG_F_BASE for d, _ in L["pre"]), "layout S: ML scratch"
        if layout == "T" and ctx == "ML":  # ... inside slots A..D
            assert all(d == NONE or 12 <= d < SIG_T_F_BASE for d, _ in L["pre"]), "layout T: ML scratch"
        if layout == "V":  # ... between slot F and the registers
            assert all(d == NONE or 12 <= d < V_F_BASE for d, _ in L["pre"]), "layout V: ML scratch"
    out = XRound(xr.nv, xr.nt, xr.np, xr.nl, lanes, xr.name, xr.np2, xr.nl2)
    out.kp, out.kl1, out.kl2 = xr.kp, xr.kl1, xr.kl2
    out.ks1, out.ks2 = xr.ks1, xr.ks2
    out.ef = xr.ef
    return out


def run_bound(rounds, mem):
    """Interprets bound rounds on a flat team memory (list of residues)."""
    for xr in rounds:
        for L in xr.lanes:
            for d, terms in L["pre"]:
                if d != NONE:
                    mem[d] = sum(k * mem[s] for s, k in terms) % P
        out = {}
        for L in xr.lanes:
            for pk, lk, dk in (("prod", "lin", "dst"), ("prod2", "lin2", "dst2")):
                if dk in L and L[dk] != NONE:
                    out[L[dk]] = (sum(mem[u] * mem[v] for u, v in L[pk])
                                  + sum(k * mem[s] for s, k in L[lk])) % P
        for d, v in out.items():
            mem[d] = v


def check_instances(X, seed=3):
    """Every bound instance computes the same as the abstract program."""
    rng = random.Random(seed)
    for name, binding, layout in ALL_INSTANCES:
        ctx = X_PROGRAMS[name]
        fb = {"S": SIG_F_BASE, "T": SIG_T_F_BASE, "V": V_F_BASE}.get(layout, F_BASE_CTX[ctx])
        rounds = [bind(xr, binding, ctx, layout) for xr in X[name]]
        mem = [rng.randrange(P) for _ in range(F_BASE + NREGS)]
        mem[fb + REG["ZERO"]] = 0
        mem[fb + REG["ONE"]] = 1
        F = {r: mem[fb + r] for r in range(NREGS)}
        A = B = None
        if binding:
            bd = list(binding) + ([binding[1]] if len(binding) == 2 else [])
            A = mem[12 * SLOTS.index(bd[1]):12 * SLOTS.index(bd[1]) + 12]
            B = mem[12 * SLOTS.index(bd[2]):12 * SLOTS.index(bd[2]) + 12]
        want_D = run_xprogram(X[name], F, A, B)
        run_bound(rounds, mem)
        if binding:
            d0 = 12 * SLOTS.index(binding[0])
            assert all(mem[d0 + e] == v for e, v in want_D.items()), f"instance {name}{binding}"
        else:
            for r, v in F.items():
                assert mem[fb + r] == v, f"instance {name} reg {r}"


# the programs k_verify_sig runs (bn256_gt.hip: the sig-only Miller loop and
# the final exponentiation); its team region ends after the last element they
# (and the hand-written helpers: registers up to FC) touch
SIG_PROGRAMS = ("SDBL", "LFEV", "FEVAL", "LINE_FIX", "MUL12", "CYC_SQR_X", "CYC_SQR",
                "SQR12_12", "LINE_FIX_12", "MUL12_12", "CYC_SQR_X_12")


def touched(bx):
    """Largest team element index a bound round reads or writes."""
    m = 0
    for L in bx.lanes:
        idx = [L["dst"], L.get("dst2", NONE)] + [d for d, _ in L["pre"]]
        idx += [s_ for _, t in L["pre"] for s_, _ in t]
        for pk, lk in (("prod", "lin"), ("prod2", "lin2")):
            idx += [u for u, v in L.get(pk, [])] + [v for u, v in L.get(pk, [])] + [s_ for s_, _ in L.get(lk, [])]
        m = max([m] + [v for v in idx if v != NONE])
    return m


def emit_x(X, path):
    sig_end = SIG_F_BASE + REG["FC.y"] + 1  # team_miller_sig's registers: ZERO .. FC
    sig_t_end = SIG_T_F_BASE + REG["FC.y"] + 1  # team_miller_sig12's: ZERO, ONE, FB, FC
    fold_end = FOLD_F_BASE + 2               # ZERO, ONE
    for name, binding, layout in ALL_INSTANCES:
        ctx = X_PROGRAMS[name]
        for xr in X[name]:
            t = touched(bind(xr, binding, ctx, layout)) + 1
            if layout == "S":
                sig_end = max(sig_end, t)
            if layout == "T":
                sig_t_end = max(sig_t_end, t)
            if ctx == "FOLD":
                fold_end = max(fold_end, t)
    sig_names = sorted({n for n, _, lay in ALL_INSTANCES if lay == "S"}, key=list(X_PROGRAMS).index)
    sig_t_names = sorted({n for n, _, lay in ALL_INSTANCES if lay == "T"}, key=list(X_PROGRAMS).index)
    v_names = sorted({n for n, _, lay in ALL_INSTANCES if lay == "V"}, key=list(X_PROGRAMS).index)
    v_end = V_F_BASE + NREGS_RUNTIME
    lines = ["// Generated by tools/gen_g2_schedule.py — do not edit.",
             "// Two-phase team programs executed by bn256_xprog.h (encoding: see there),",
             "// one table per call-site instance (absolute team element indices).",
             "#pragma once", "#include <stdint.h>", "namespace hg {",
             f"// HG_P2N: ({NEG_MULT}p)'' (the negation constant of pre-pass and linear terms)",
             "#define HG_P2N " + ", ".join("0x%08xu" % v for v in P2N),
             "enum XProg { " + ", ".join([f"XP_{n}" for n in X_PROGRAMS] + [f"XP_{n}_S" for n in sig_names]
                                         + [f"XP_{n}_T" for n in sig_t_names]
                                         + [f"XP_{n}_V" for n in v_names]) + " };",
             f"static constexpr int kXFetchWords = {X_FETCH_WORDS};",
             f"static constexpr int kFoldRegBase = {FOLD_F_BASE};  // FOLD team region: ZERO, ONE here",
             f"static constexpr int kFoldTeamElems = {fold_end + fold_end % 2};  // elements the fold programs touch",
             f"static constexpr int kSigRegBase = {SIG_F_BASE};  // k_verify_sig's layout S: registers here",
             f"static constexpr int kSigTeamElems = {sig_end + sig_end % 2};  // k_verify_sig's team region (layout S)",
             f"static constexpr int kSigTRegBase = {SIG_T_F_BASE};  // k_verify_sig12's layout T: registers here",
             f"static constexpr int kSigTTeamElems = {sig_t_end + sig_t_end % 2};  // k_verify_sig12's team region",
             f"static constexpr int kVRegBase = {V_F_BASE};  // k_verify_ml's layout V: registers here",
             f"static constexpr int kVTeamElems = {v_end + v_end % 2};  // k_verify_ml's team region",
             "template <int PROG, int D = -1, int A = -1, int B = -1> struct XInst;"]
    words = []
    for name, binding, layout in ALL_INSTANCES:
        ctx = X_PROGRAMS[name]
        rounds = []
        for xr in X[name]:
            bx = bind(xr, binding, ctx, layout)
            off = len(words)
            for t in range(16):
                hv = bx.lane_halves(t)
                words += [hv[2 * w] | (hv[2 * w + 1] << 16) for w in range(bx.words())]
            assert bx.words() <= X_FETCH_WORDS, f"{name}: round wider than the prefetch"
            rounds.append((bx, off))
        calls = []
        for i, (bx, off) in enumerate(rounds):
            # each round prefetches the next round's words (the last one: the caller's hint)
            nxt = f"XHint{{{rounds[i + 1][1]}, {rounds[i + 1][0].words()}}}" if i + 1 < len(rounds) else "h"
            lz = int(name in LAZY_PROGRAMS and bx.nl > 0)
            assert not (lz and bx.fused), "a lazy round is not fused"
            # FU: REDC interleaved with the last product (bn256_xprog.h x_job):
            # the final exponentiation's and the sig-only Miller loop's rounds;
            # not the GT fold's (several waves per SIMD hide the chain), not
            # two-job rounds, not the pk-side G2 steps (measured: config 2
            # 0.5 % slower with them, profiles/r03fuse_redc_ab.json)
            fu = int(not bx.fused and (ctx == "FE" or name in SIG_PROGRAMS))
            calls.append(f"x_round<{bx.nv}, {bx.nt}, {bx.np}, {bx.nl}, {bx.words()}, {bx.np2}, {bx.nl2}, "
                         f"{bx.kp}, {bx.kl1}, {bx.kl2}, {bx.ks1}, {bx.ks2}, {lz}, {bx.ef}, {fu}>(T, S, {off}, {nxt});")
        args = ", ".join(f"S_{b}" for b in binding)
        targs = f"XP_{name}{'_' + layout if layout else ''}" + (", " + args if args else "")
        lines.append(f"template <> struct XInst<{targs}> {{ static constexpr int kOff = {rounds[0][1]}, "
                     f"kW = {rounds[0][0].words()}; HG_DEV static void run(const Team& T, XStream& S, XHint h) {{ "
                     + " ".join(calls) + " } };")
    words += [0] * X_FETCH_WORDS  # a prefetch reads X_FETCH_WORDS words from any lane's block
    lines.insert(9, f"__constant__ static const uint32_t kXTab[{len(words)}] = {{")
    tab = []
    for i in range(0, len(words), 12):
        tab.append("  " + ", ".join("0x%08xu" % w for w in words[i:i + 12]) + ",")
    tab.append("};")
    lines[10:10] = tab
    lines.append("}  // namespace hg")
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")
    return len(words)


# ------------------------------------------------------------------ emit
def emit(path):
    lines = ["// Generated by tools/gen_g2_schedule.py — do not edit.",
             "// Lane-parallel team programs (see the generator for the encoding).",
             "#pragma once", "#include <stdint.h>", "namespace hg {",
             f"static constexpr int kG2Regs = {NREGS_RUNTIME};  // the kernels' register file",
             f"static constexpr int kG2RegsAll = {NREGS};  // + the Jacobian cross-check programs' registers",
             f"static constexpr int kG2MaxSlots = {MAX_NSLOT};",
             f"static constexpr int kG2MaxTerms = {MAX_TERMS};", f"static constexpr uint8_t kG2None = {NONE};",
             f"static constexpr int kOpSlotA = {SLOT_A};", f"static constexpr int kOpSlotB = {SLOT_B};"]
    for k, v in REG.items():
        if v < 128:
            lines.append(f"static constexpr int R_{k.replace('.', '_')} = {v};")
    lines.append(f"struct G2Lane {{\n  uint8_t dst, pad[3];\n  uint8_t ar[{MAX_NSLOT}][{MAX_TERMS}];\n"
                 f"  int8_t ac[{MAX_NSLOT}][{MAX_TERMS}];\n  uint8_t br[{MAX_NSLOT}][{MAX_TERMS}];\n"
                 f"  int8_t bc[{MAX_NSLOT}][{MAX_TERMS}];\n}};")
    lines.append(f"struct G2Round {{\n  int nslot, nta[{MAX_NSLOT}], ntb[{MAX_NSLOT}], first;  // first = index into kG2Lanes\n}};")
    all_lanes = []
    rounds = {}
    for name, prog in PROGRAMS.items():
        if name not in LEGACY:
            continue
        rounds[name] = []
        for r in prog:
            nslot = max(len(l.slots) for l in r)
            nta = [max((len(l.slots[s][0]) if s < len(l.slots) else 0) for l in r) for s in range(MAX_NSLOT)]
            ntb = [max((len(l.slots[s][1]) if s < len(l.slots) else 0) for l in r) for s in range(MAX_NSLOT)]
            rounds[name].append((nslot, nta, ntb, len(all_lanes)))
            for t in range(16):
                l = r[t] if t < len(r) else None
                ent = {"dst": l.dst if l else NONE, "ar": [], "ac": [], "br": [], "bc": []}
                for s in range(MAX_NSLOT):
                    a, b = (l.slots[s] if (l and s < len(l.slots)) else ([], []))
                    pa = list(a) + [(REG["ZERO"], 0)] * (MAX_TERMS - len(a))
                    pb = list(b) + [(REG["ZERO"], 0)] * (MAX_TERMS - len(b))
                    ent["ar"].append([x for x, _ in pa])
                    ent["ac"].append([k for _, k in pa])
                    ent["br"].append([x for x, _ in pb])
                    ent["bc"].append([k for _, k in pb])
                all_lanes.append(ent)

    def arr(v):
        return "{" + ", ".join(arr(x) if isinstance(x, list) else str(x) for x in v) + "}"

    lines.append(f"__constant__ static const G2Lane kG2Lanes[{len(all_lanes)}] = {{")
    for e in all_lanes:
        lines.append(f"  {{{e['dst']}, {{0, 0, 0}}, {arr(e['ar'])}, {arr(e['ac'])}, {arr(e['br'])}, {arr(e['bc'])}}},")
    lines.append("};")
    for name, rs in rounds.items():
        body = ", ".join(f"{{{n}, {arr(a)}, {arr(b)}, {f}}}" for n, a, b, f in rs)
        lines.append(f"static constexpr int kProg{name}Len = {len(rs)};")
        lines.append(f"static constexpr G2Round kProg{name}[{len(rs)}] = {{{body}}};")
    lines.append("}  // namespace hg")
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    validate()
    csrc = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "handel_amd", "csrc")
    emit(os.path.join(csrc, "bn256_g2sched.h"))
    Xp = validate_x()
    check_instances(Xp)
    nwords = emit_x(Xp, os.path.join(csrc, "bn256_xtab.h"))
    print(len(ALL_INSTANCES), "instances,", nwords * 4, "table bytes")
    for name, rounds in Xp.items():
        print(name, [(r.nv, r.nt, r.np, r.nl, r.words()) for r in rounds])
    print("validated and wrote bn256_g2sched.h, bn256_xtab.h")
