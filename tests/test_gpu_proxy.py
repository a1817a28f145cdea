"""GPU suite: the config-4 process-model proxy (tests/native/handel_proxy.c).

P processes, each with its own context and a launch-merging hg_batcher, K
Handel instances per process checking one multisignature at a time
(simul/node/main.go:63-131, processing.go:228-287). A small run must give the
expected verdict for every check (every 8th aggregate tampered), and process
0's requests and verdicts are checked against the C restatement of the
reference here.
"""

import json
import os
import subprocess

import numpy as np
import pytest

from handel_amd import build as B
from handel_amd.engine import REQ_DTYPE
from oracle import ref_lib as R
from tests import _fixtures as F

pytestmark = pytest.mark.gpu


def _run(tmp, *args):
    exe = B.build_proxy(verbose=False)
    cmd = [exe, B.LIB, *map(str, args), "-d", str(tmp)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-2000:])
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("level", [0, 2])
def test_proxy_verdicts_match_oracle(tmp_path, level):
    out = _run(tmp_path, "-p", 2, "-k", 24, "-n", 300, "-r", 5, "-w", 4, "-L", level, "-P", 1)
    assert out["mismatches"] == 0 and out["requests"] == 2 * 24 * 5
    assert out["tables_after"] == level
    assert out["mean_batch"] >= 1.0
    reg = (tmp_path / "reg.bin").read_bytes()
    reqs = np.frombuffer((tmp_path / "reqs.bin").read_bytes(), dtype=REQ_DTYPE)
    words = np.frombuffer((tmp_path / "words.bin").read_bytes(), dtype=np.uint64)
    sigs = (tmp_path / "sigs.bin").read_bytes()
    got = np.frombuffer((tmp_path / "codes.bin").read_bytes(), dtype=np.int32)
    want = R.verify_aggregate(F.LIB_MESSAGE, reg, reqs["offset"], reqs["bitlen"], reqs["level_size"], words,
                              reqs["word_offset"].astype(np.uint64), sigs, nthreads=8)
    assert np.array_equal(got, want)
    assert (got == 1).sum() == (len(got) + 7) // 8  # exactly the tampered eighth


def test_proxy_batches_merge_concurrent_instances(tmp_path):
    """With many instances per process the batcher merges their checks: far
    fewer GPU batches than checks."""
    out = _run(tmp_path, "-p", 1, "-k", 64, "-n", 128, "-r", 4, "-w", 8, "-L", 2, "-P", 1)
    assert out["mismatches"] == 0
    assert out["batches"] < out["requests"] // 4
