"""GPU suite: the RCCL branch of the N-rank bench, run on the one GPU a test
box has, so that the first RCCL execution is not the
driver's 8-GPU scaling run.

bench.py with HG_BENCH_FORCE_PG=1 takes the multi-rank path at world size 1:
init_process_group("nccl", device_id=cuda:0), four lanes in flight, each
lane's verdict bitset all-gathered over RCCL on the lane's own stream
(torch.cuda.ExternalStream of hg_lane_stream), the timer's barriers and
max-over-ranks all_gather, the prewarm's all_reduce; bench itself asserts
every lane's gathered bitset against the expected verdicts (1/8 tampered)
before it prints its line. SURVEY.md §8(e).
"""

import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_rccl_branch_world_one():
    env = {k: v for k, v in os.environ.items() if k not in ("HG_BENCH_BACKEND", "HG_BENCH_LAUNCHED")}
    env.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()),
               HG_BENCH_FORCE_PG="1")
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--steps", "4", "--warmup", "1",
                        "--prewarm", "0.05", "--no-extra", "--no-cpu"],
                       capture_output=True, text=True, timeout=280, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    g = line["gather"]
    assert g["backend"] == "nccl" and g["world_size_seen"] == 1
    assert g["lanes_checked"] == 4 and line["batches_in_flight"] == 4
    assert line["n_gpus"] == 1 and line["value"] > 0
