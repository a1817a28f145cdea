"""The sig-only pairing kernels' final exponentiation on layout S
(bn256_sigfe.h SigFE::team_final_exp_fc_s and SigFE::t12_pow_v_s, shared by
k_verify_sig and k_verify_sig12): the chain runs over seven Fp12 slots, with
several slots reused for different values along the way.

This test reads the two device functions' text, turns their statements into
operations on a slot dictionary (Fp12 values from the oracle) and runs them:
the value left in slot F must be oracle.final_exponentiation_fc(f), so a slot
overwritten while still needed shows up here, not only on the GPU. The team
programs themselves (one table per call-site instance, layout S) are checked
by tools/gen_g2_schedule.py check_instances (tests/test_g2_schedule.py).
"""

import os
import random
import re

from oracle import bn256_oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "handel_amd", "csrc")
V = 1868033  # u = v^3 (bn256_xprog.h t12_pow_v_x)


def _body(path, signature):
    src = open(path).read()
    i = src.index(signature)
    i = src.index("{", i)
    depth, j = 0, i
    while True:
        if src[j] == "{":
            depth += 1
        elif src[j] == "}":
            depth -= 1
            if depth == 0:
                return src[i + 1:j]
        j += 1


def _to_python(body):
    """The C++ subset these functions use -> Python source."""
    body = re.sub(r"//[^\n]*", "", body)
    body = re.sub(r"#pragma[^\n]*", "", body)
    # drop the prefetch hints (declarations spanning lines up to ';')
    body = re.sub(r"const XHint \w+ = [^;]*;", "", body, flags=re.S)
    body = re.sub(r"static_assert\([^;]*;", "", body, flags=re.S)
    body = re.sub(r"const int nsq\[4\] = \{([^}]*)\};", r"nsq = [\1]", body)
    body = re.sub(r"const XHint mul = [^;]*;", "", body, flags=re.S)
    out, depth = [], 0
    for raw in body.replace("{", "{\n").replace("}", "\n}\n").split("\n"):
        line = raw.strip()
        if not line:
            continue
        if line == "}":
            depth -= 1
            continue
        if line.startswith("} else"):
            depth -= 1
            line = line[1:].strip()

        def stmt(s):
            s = s.strip().rstrip(";")
            m = re.match(r"t12_(conj|frob|frob2|copy)\(T, S_(\w), S_(\w)\)$", s)
            if m:
                return f"{m.group(1)}('{m.group(2)}', '{m.group(3)}')"
            m = re.match(r"t12_park\(T, S_(\w), park\((\d)\)\)$", s)
            if m:
                return f"park('{m.group(1)}', {m.group(2)})"
            m = re.match(r"t12_unpark\(T, S_(\w), park\((\d)\)\)$", s)
            if m:
                return f"unpark('{m.group(1)}', {m.group(2)})"
            m = re.match(r"t12_inv_norm\(T, S_(\w)\)$", s)
            if m:
                return f"inv('{m.group(1)}')"
            m = re.match(r"(IMul12S|IMul12)<S_(\w), S_(\w), S_(\w)>::run\(.*\)$", s)
            if m:
                return f"mul('{m.group(2)}', '{m.group(3)}', '{m.group(4)}')"
            m = re.match(r"(ICycS|ICyc0S)<S_(\w), S_(\w)>::run\(.*\)$", s)
            if m:
                return f"sqr('{m.group(2)}', '{m.group(3)}')"
            if s == "handover()":
                return s
            m = re.match(r"t12_pow_v_s<S_(\w), S_(\w), S_(\w)>\(.*\)$", s)
            if m:
                return f"powv('{m.group(1)}', '{m.group(2)}', '{m.group(3)}')"
            m = re.match(r"(IMul12S|ICycS)<D, (\w+)(, (\w+))?>::run\(.*\)$", s)
            if m:  # inside t12_pow_v_s: template slots D, SA, SK
                return f"{'mul' if m.group(1) == 'IMul12S' else 'sqr'}(D, {m.group(2)}" + (
                    f", {m.group(4)})" if m.group(4) else ")")
            m = re.match(r"t12_conj\(T, (\w+), (\w+)\)$", s)
            if m:
                return f"conj({m.group(1)}, {m.group(2)})"
            if s.startswith("nsq ="):
                return s
            raise ValueError(f"unhandled statement: {s!r}")

        ind = "    " * depth
        m = re.match(r"for \(int (\w+) = 0; \w+ < ([^;]+); \w+\+\+\) \{$", line)
        if m:
            out.append(f"{ind}for {m.group(1)} in range({m.group(2)}):")
            depth += 1
            continue
        m = re.match(r"for \(int (\w+) = 0; \w+ < ([^;]+); \w+\+\+\) (.+;)$", line)
        if m:
            out.append(f"{ind}for {m.group(1)} in range({m.group(2)}):")
            out.append(f"{ind}    {stmt(m.group(3))}")
            continue
        m = re.match(r"(else )?if \((.*)\) \{$", line)
        if m:
            cond = m.group(2).replace("&&", "and").replace("||", "or")
            out.append(f"{ind}{'elif' if m.group(1) else 'if'} {cond}:")
            depth += 1
            continue
        if line == "else {":
            out.append(f"{ind}else:")
            depth += 1
            continue
        m = re.match(r"if \(((?:[^()]|\([^()]*\))*)\) (.+;)$", line)
        if m:
            out.append(f"{ind}if {m.group(1)}:")
            out.append(f"{ind}    {stmt(m.group(2))}")
            continue
        m = re.match(r"else (.+;)$", line)
        if m:
            out.append(f"{ind}else:")
            out.append(f"{ind}    {stmt(m.group(1))}")
            continue
        out.append(ind + stmt(line))
    return "\n".join(out)


import pytest  # noqa: E402

SIGFE = os.path.join(CSRC, "bn256_sigfe.h")


def _t_parts():
    """layout T's chain in its two parts (fe_t_norm: up to the norm N in B;
    fe_t_rest: from N^-1 in B on), as the split kernels run them."""
    return _body(SIGFE, "HG_DEV static void fe_t_norm("), _body(SIGFE, "HG_DEV static void fe_t_rest(")


def _fc_source(layout):
    body = _body(SIGFE, f"HG_DEV static void team_final_exp_fc_{layout}(")
    if layout == "t":  # the monolithic kernel calls the two parts around t12_inv_norm
        norm, rest = _t_parts()
        body = re.sub(r"fe_t_norm\(T, S, [^;]*\);", lambda m: norm, body)
        assert "fe_t_rest(T, S, park);" in body
        body = body.replace("fe_t_rest(T, S, park);", rest)
    return _to_python(body)


@pytest.mark.parametrize("layout,slots_used,split", [("s", "FABCDEG", False), ("t", "FABCD", False),
                                                     ("t", "FABCD", True)])
def test_final_exp_layout_matches_oracle(layout, slots_used, split):
    """layout s: k_verify_sig's seven slots; layout t: k_verify_sig12's five
    slots, two values parked in HBM (t12_park / t12_unpark). split: the
    three-kernel form (bn256_sig12.hip k_sig12_miller / k_sig12_fe): fe_t_norm
    in the first kernel, then a fresh team region in the last one holding only
    what k_sig12_fe rebuilds — f in F, conj(f) in D, N^-1 in B (from the
    handed-over terms and the batched inverse), garbage in every other slot —
    and fe_t_rest from there."""
    if split:
        norm, rest = _t_parts()
        fc_src = _to_python(norm) + "\nhandover()\n" + _to_python(rest)
    else:
        fc_src = _fc_source(layout)
    pow_src = _to_python(_body(SIGFE, "HG_DEV static void t12_pow_v_s("))
    rng = random.Random(5)
    f = [(rng.randrange(O.P), rng.randrange(O.P)) for _ in range(6)]
    slots = {}

    def conj(d, a):
        slots[d] = O.f12_conj(slots[a])

    def frob(d, a):
        slots[d] = O.f12_frob(slots[a])

    def frob2(d, a):
        slots[d] = O.f12_frob2(slots[a])

    def copy(d, a):
        slots[d] = slots[a]

    def inv(d):
        slots[d] = O.f12_inv(slots[d])

    def mul(d, a, b):
        slots[d] = O.f12_mul(slots[a], slots[b])

    def sqr(d, a):
        slots[d] = O.f12_sqr(slots[a])

    parked = {}

    def park(a, k):
        parked[k] = slots[a]

    def unpark(d, k):
        slots[d] = parked.pop(k)  # read once, after it was written

    env = {"conj": conj, "frob": frob, "frob2": frob2, "copy": copy, "inv": inv, "mul": mul, "sqr": sqr,
           "park": park, "unpark": unpark}

    def powv(d, sa, sk):
        assert len({d, sa, sk}) == 3
        loc = dict(env, D=d, SA=sa, SK=sk)
        exec(pow_src, loc)
        assert slots[d] == O.f12_pow(slots[sa], V), "t12_pow_v_s"

    env["powv"] = powv

    def handover():
        n_inv = O.f12_inv(slots["B"])
        f_val = slots["F"]
        for s in slots_used:  # a new kernel's team region
            slots[s] = O.f12_pow(f, rng.randrange(2, 1000))
        slots["F"] = f_val
        slots["D"] = O.f12_conj(f_val)
        slots["B"] = n_inv

    env["handover"] = handover
    for s in slots_used:  # garbage everywhere but F
        slots[s] = O.f12_pow(f, rng.randrange(2, 1000)) if s != "F" else f
    exec(fc_src, dict(env))
    assert set(slots) == set(slots_used), f"layout {layout} uses slots {slots_used} only"
    assert not parked, "every parked value is taken back"
    assert slots["F"] == O.final_exponentiation_fc(f)
