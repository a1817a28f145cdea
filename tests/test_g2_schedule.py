"""CPU suite: the generated team programs (tools/gen_g2_schedule.py, the
tables compiled into the HIP library) compute exactly x/crypto's
lineFunctionDouble / lineFunctionAdd and the Fp12 squarings; and the
committed header is the one the generator emits."""

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import gen_g2_schedule as G  # noqa: E402


def test_schedule_interpreter_matches_oracle():
    assert G.validate(seed=11)


def test_committed_header_is_current(tmp_path):
    out = tmp_path / "sched.h"
    G.emit(str(out))
    committed = os.path.join(ROOT, "handel_amd", "csrc", "bn256_g2sched.h")
    with open(committed) as f:
        assert f.read() == out.read_text()


def test_round_bounds():
    for name, prog in G.PROGRAMS.items():
        for i, r in enumerate(prog):
            worst = G.check_round(r, f"{name}[{i}]")
            assert worst / G.R_OVER_P + 1 < 8
