"""CPU suite: the generated team programs (tools/gen_g2_schedule.py, the
tables compiled into the HIP library) compute exactly x/crypto's
lineFunctionDouble / lineFunctionAdd and the Fp12 products/squarings; and the
committed headers are the ones the generator emits."""

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import gen_g2_schedule as G  # noqa: E402

CSRC = os.path.join(ROOT, "handel_amd", "csrc")


def test_schedule_interpreter_matches_oracle():
    assert G.validate(seed=11)


def test_two_phase_programs_match_oracle():
    # validate_x checks every compiled round against the oracle's line
    # functions and Fp12 ops, including the column / REDC-input bounds
    X = G.validate_x(seed=5)
    G.check_instances(X, seed=7)


def test_committed_headers_are_current(tmp_path):
    out = tmp_path / "sched.h"
    G.emit(str(out))
    with open(os.path.join(CSRC, "bn256_g2sched.h")) as f:
        assert f.read() == out.read_text()
    outx = tmp_path / "xtab.h"
    G.emit_x(G.compile_all(), str(outx))
    with open(os.path.join(CSRC, "bn256_xtab.h")) as f:
        assert f.read() == outx.read_text()


def test_round_bounds():
    # single-phase table format (bn256_g2sched.h): slot/term/product bounds
    for name in G.LEGACY:
        for i, r in enumerate(G.PROGRAMS[name]):
            worst = G.check_round(r, f"{name}[{i}]")
            assert worst / G.R_OVER_P + 1 < 8
