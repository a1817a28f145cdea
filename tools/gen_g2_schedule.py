#!/usr/bin/env python3
"""Generates handel_amd/csrc/bn256_g2sched.h: the lane-parallel schedule of the
Miller loop's G2 steps (x/crypto optate.go lineFunctionDouble /
lineFunctionAdd) for a 16-lane team.

A *program* is a short list of rounds. In a round every lane of the team
computes one Fp element
    dst = sum_{slot} (sum_m ca_m * F[ra_m]) * (sum_m cb_m * F[rb_m])
over the team's LDS register file F (Fp elements in Montgomery form), with
small signed integer coefficients, then stores it. All lanes run the same
instruction stream (only addresses and coefficients differ), rounds are
separated by a team barrier. The tables are validated here by interpreting
them with plain modular arithmetic against the oracle's line functions
(tests/test_g2_schedule.py runs the same check in the CPU suite).

Build tooling only: nothing in the product imports this file.
"""

from __future__ import annotations

import os
import random
import sys

P = 65000549695646603732796438742359905742825358107623003571877145026864184071783
# R/p for the 10 x 26-bit Montgomery representation: REDC(T) < T/R + p
R_OVER_P = (1 << 260) / P
MAX_NSLOT = 3
MAX_TERMS = 6

# ------------------------------------------------------------------ register file
FP_SCALARS = ["ZERO", "ONE", "PX", "PY", "SX", "NSY"]
FP2_REGS = ["X", "Y", "Z", "T", "QX", "QY", "NQY", "R2", "P1X", "P1Y", "P1R2", "P2X",
            "FA", "FBX", "FCY", "FB", "FC", "LA", "LB", "LC", "F2ONE", "F2ZERO",
            # doubling temporaries
            "A", "B", "S", "C", "W", "G", "V", "ET", "ZP", "TPY",
            # addition temporaries
            "AB", "S1", "D", "I", "S2", "H", "J", "AV", "L1", "XN", "YJ", "TP", "LA1", "S3"]
REG = {}
for i, n in enumerate(FP_SCALARS):
    REG[n] = i
_base = len(FP_SCALARS)
for i, n in enumerate(FP2_REGS):
    REG[n + ".x"] = _base + 2 * i
    REG[n + ".y"] = _base + 2 * i + 1
NREGS = _base + 2 * len(FP2_REGS)
NONE = 255


def comp(name, c):
    return REG[f"{name}.{c}"]


# ------------------------------------------------------------------ expression helpers
# An Fp2 linear combination is a list of (fp2_name, coef). Its component c is
# the Fp lincomb [(reg(name.c), coef)].
def fp2_comp(lc, c):
    return [(comp(n, c), k) for n, k in lc]


def neg(terms):
    return [(r, -k) for r, k in terms]


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


# ------------------------------------------------------------------ programs
def fixed_line_eval():
    # FB = FBX * SX, FC = FCY * NSY  (the G2Base line at -sig)
    return smul("FB", [("FBX", 1)], "SX") + smul("FC", [("FCY", 1)], "NSY")


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


PROGRAMS = {
    "DBL": prog_double(),
    "ADD_POS": prog_add("QX", "QY", "R2"),
    "ADD_NEG": prog_add("QX", "NQY", "R2"),
    "ADD_F1": prog_add("P1X", "P1Y", "P1R2"),
    "ADD_F2": prog_add("P2X", "QY", "R2"),
}


# ------------------------------------------------------------------ checks + interpreter
def bound(terms):
    return sum(abs(k) for _, k in terms)


def check_round(lanes, name):
    assert len(lanes) <= 16, f"{name}: {len(lanes)} lanes"
    dsts = [l.dst for l in lanes]
    assert len(set(dsts)) == len(dsts), f"{name}: duplicate destinations"
    total = 0
    for l in lanes:
        assert len(l.slots) <= MAX_NSLOT, f"{name}: too many slots"
        t = 0
        for a, b in l.slots:
            assert len(a) <= MAX_TERMS and len(b) <= MAX_TERMS, f"{name}: too many terms {a} {b}"
            t += bound(a) * bound(b)
        # REDC output < (t / R_OVER_P + 1) p must stay below 8p (fp_reduce8)
        assert t / R_OVER_P + 1 < 8, f"{name}: product bound {t}"
        total = max(total, t)
    # a round must not read a register another lane of the same round writes
    reads = {r for l in lanes for a, b in l.slots for r, _ in a + b}
    clash = reads & set(dsts)
    assert not clash, f"{name}: read/write clash on {[k for k, v in REG.items() if v in clash]}"
    return total


def run_program(prog, F):
    """Interprets a program on a register file of plain residues mod p."""
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
        for i, r in enumerate(prog):
            check_round(r, f"{name}[{i}]")
    for trial in range(4):
        Q = O.g2_mul(O.G2_GEN, rng.randrange(1, O.ORDER))
        Hp = O.g1_mul(O.G1_GEN, rng.randrange(1, O.ORDER))
        Rj = O.jac_mul(O.FP2_OPS, O.to_jac(O.FP2_OPS, Q), rng.randrange(2, 1000))
        r = (Rj[0], Rj[1], Rj[2], O.f2_sqr(Rj[2]))
        F = {i: rng.randrange(P) for i in range(NREGS)}
        F[REG["ZERO"]] = 0
        F[REG["ONE"]] = 1
        F[REG["PX"]], F[REG["PY"]] = Hp

        def put(n, v):
            F[comp(n, "x")], F[comp(n, "y")] = v

        def get(n):
            return (F[comp(n, "x")], F[comp(n, "y")])

        for n, v in zip(("X", "Y", "Z", "T"), r):
            put(n, v)
        put("QX", Q[0])
        put("QY", Q[1])
        put("NQY", O.f2_neg(Q[1]))
        put("R2", O.f2_sqr(Q[1]))
        a, b, c, r_new = O._line_double(r, *Hp)
        G = run_program(PROGRAMS["DBL"], dict(F))
        assert [(G[comp(n, "x")], G[comp(n, "y")]) for n in ("X", "Y", "Z", "T")] == list(r_new), "DBL point"
        assert (G[comp("LA", "x")], G[comp("LA", "y")]) == a, "DBL a"
        assert (G[comp("LB", "x")], G[comp("LB", "y")]) == b, "DBL b"
        assert (G[comp("LC", "x")], G[comp("LC", "y")]) == c, "DBL c"
        for prog, pq in (("ADD_POS", (Q[0], Q[1])), ("ADD_NEG", (Q[0], O.f2_neg(Q[1])))):
            a, b, c, r_new = O._line_add(r, pq, *Hp, O.f2_sqr(pq[1]))
            G = run_program(PROGRAMS[prog], dict(F))
            assert [(G[comp(n, "x")], G[comp(n, "y")]) for n in ("X", "Y", "Z", "T")] == list(r_new), prog
            assert [(G[comp(n, "x")], G[comp(n, "y")]) for n in ("LA", "LB", "LC")] == [a, b, c], prog + " line"
    return True


# ------------------------------------------------------------------ emit
def emit(path):
    lines = ["// Generated by tools/gen_g2_schedule.py — do not edit.",
             "// Lane-parallel schedule of the Miller loop's G2 steps (see the generator).",
             "#pragma once", "#include <stdint.h>", "namespace hg {",
             f"static constexpr int kG2Regs = {NREGS};", f"static constexpr int kG2MaxSlots = {MAX_NSLOT};",
             f"static constexpr int kG2MaxTerms = {MAX_TERMS};", f"static constexpr uint8_t kG2None = {NONE};"]
    for k, v in REG.items():
        lines.append(f"static constexpr int R_{k.replace('.', '_')} = {v};")
    lines.append("struct G2Lane {\n  uint8_t dst, pad[3];\n  uint8_t ar[3][6];\n  int8_t ac[3][6];\n"
                 "  uint8_t br[3][6];\n  int8_t bc[3][6];\n};")
    lines.append("struct G2Round {\n  int nslot, nta[3], ntb[3], first;  // first = index into kG2Lanes\n};")
    all_lanes = []
    rounds = {}
    for name, prog in PROGRAMS.items():
        rounds[name] = []
        for r in prog:
            nslot = max(len(l.slots) for l in r)
            nta = [max((len(l.slots[s][0]) if s < len(l.slots) else 0) for l in r) for s in range(3)]
            ntb = [max((len(l.slots[s][1]) if s < len(l.slots) else 0) for l in r) for s in range(3)]
            rounds[name].append((nslot, nta, ntb, len(all_lanes)))
            for t in range(16):
                l = r[t] if t < len(r) else None
                ent = {"dst": l.dst if l else NONE, "ar": [], "ac": [], "br": [], "bc": []}
                for s in range(3):
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
        body = ", ".join(f"{{{n}, {{{a[0]}, {a[1]}, {a[2]}}}, {{{b[0]}, {b[1]}, {b[2]}}}, {f}}}" for n, a, b, f in rs)
        lines.append(f"static constexpr int kProg{name}Len = {len(rs)};")
        lines.append(f"static constexpr G2Round kProg{name}[{len(rs)}] = {{{body}}};")
    lines.append("}  // namespace hg")
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    validate()
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "handel_amd", "csrc", "bn256_g2sched.h")
    emit(out)
    print("validated and wrote", os.path.normpath(out))
