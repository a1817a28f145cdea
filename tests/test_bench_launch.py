"""CPU suite: bench.py's multi-GPU entry as the driver invokes it.

`python bench.py --gpus N` (no torchrun around it) must become an N-rank run,
one process per GPU, started before any HIP call; a world that differs from
--gpus must fail instead of printing a line with the wrong n_gpus; and the
one-GPU-only config-4 proxy line must stay off every multi-rank run
(SURVEY.md §8(e)). The launch is exercised for real here
with the gloo backend and no device (--launch-probe).
"""

import argparse
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                             "MASTER_PORT", "HG_BENCH_LAUNCHED")}
    env.update(kw)
    return env


@pytest.mark.parametrize("n", [2, 3])
def test_gpus_n_launches_n_ranks(n):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--launch-probe"],
                       capture_output=True, text=True, timeout=240, env=_env(HG_BENCH_BACKEND="gloo"))
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert out == {"n_gpus": n, "world_size_seen": n, "ranks": list(range(n)), "launched": True}


def test_gpus_one_runs_in_process():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--launch-probe"],
                       capture_output=True, text=True, timeout=240, env=_env())
    assert r.returncode == 0, r.stderr[-3000:]
    assert json.loads(r.stdout.strip().splitlines()[-1]) == {"n_gpus": 1, "world_size_seen": 1, "ranks": [0],
                                                             "launched": False}


def test_world_size_mismatch_exits_nonzero():
    # a launcher that started one rank while --gpus asks for two
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--launch-probe"],
                       capture_output=True, text=True, timeout=240,
                       env=_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"))
    assert r.returncode == 2 and "--gpus 2" in r.stderr


def test_config4_proxy_only_on_a_one_rank_run():
    sys.path.insert(0, ROOT)
    import bench

    def a(**kw):
        d = dict(no_service=False, no_extra=False)
        d.update(kw)
        return argparse.Namespace(**d)

    assert bench.want_config4_proxy(0, 1, a())
    assert not bench.want_config4_proxy(0, 2, a())
    assert not bench.want_config4_proxy(1, 2, a())
    assert not bench.want_config4_proxy(0, 1, a(no_service=True))
    assert not bench.want_config4_proxy(0, 1, a(no_extra=True))
    # the line's assignment sits under the guard (the r04 regression: only
    # progress() was guarded)
    src = open(os.path.join(ROOT, "bench.py")).read()
    i = src.index("if want_config4_proxy(rank, world, args):")
    j = src.index('extra["config4_proxy"]')
    assert i < j and "\n        extra" not in src[i:j] and src[j - 12:j] == " " * 12


@pytest.mark.parametrize("n", [1, 2])
def test_cpu_baseline_on_every_world_size(n):
    """an N-rank line carries `cpu_baseline` too (rank 0
    runs it after the timed regions, the other ranks wait at a barrier;
    bench.cpu_baseline_on_rank0, the function main() uses). Exercised through
    the real launcher with gloo and the CPU oracle on a tiny workload."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--cpu-probe"],
                       capture_output=True, text=True, timeout=300, env=_env(HG_BENCH_BACKEND="gloo"))
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["n_gpus"] == n
    cpu = out["cpu_baseline"]
    assert "error" not in cpu, cpu
    assert cpu["value"] > 0 and cpu["cores"] >= 1 and cpu["kind"] == "port" and cpu["sample"]
    # the same call site serves the headline and config 2's lines at any world
    src = open(os.path.join(ROOT, "bench.py")).read()
    assert "world == 1 and not args.no_cpu" not in src
    assert src.count("cpu_baseline_on_rank0(") >= 3
