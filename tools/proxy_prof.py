#!/usr/bin/env python3
"""Why the contexts-model proxy stalls under rocprofv3.

  python3 tools/proxy_prof.py OUTDIR [procs ...]

Runs tests/native/handel_proxy.c's contexts model (-D 0: every process forks
from a parent that never touched the GPU, then opens its own context) under
`rocprofv3 --kernel-trace` with 1, 2, ... processes, each run in a session of
its own with a time limit: on a timeout the whole process group is killed
(the proxy's forked children included) and the series stops there. Every
process reports its phases on stderr (handel_proxy.c stage()), so the
record says which phase each child reached. Writes OUTDIR/proxy_prof.json.
This script never touches the GPU itself.
"""

import json
import os
import signal
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from handel_amd import build as B  # noqa: E402


def one(out, procs, timeout, profiled):
    d = os.path.join(out, f"p{procs}{'' if profiled else '_plain'}")
    os.makedirs(d, exist_ok=True)
    cmd = [B.HANDEL_PROXY, B.LIB, "-D", "0", "-P", "1", "-p", str(procs)]
    if profiled:
        cmd = ["rocprofv3", "--kernel-trace", "-d", os.path.join(d, "kt"), "-o", "run", "--", *cmd]
    t0 = time.time()
    pr = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, start_new_session=True)
    try:
        so, se = pr.communicate(timeout=timeout)
        rc, timed_out = pr.returncode, False
    except subprocess.TimeoutExpired:
        os.killpg(pr.pid, signal.SIGKILL)
        so, se = pr.communicate()
        rc, timed_out = None, True
    rec = {"procs": procs, "profiled": profiled, "rc": rc, "timed_out": timed_out,
           "wall_s": round(time.time() - t0, 2), "stages": [ln for ln in se.splitlines() if ln.startswith("[proxy")],
           "stderr_other": [ln for ln in se.splitlines() if not ln.startswith("[proxy")][-15:]}
    try:
        rec["line"] = json.loads(so.strip().splitlines()[-1])
    except (ValueError, IndexError):
        rec["stdout_tail"] = so[-300:]
    return rec


def main():
    out = sys.argv[1]
    series = [int(x) for x in sys.argv[2:]] or [1, 2, 8]
    os.makedirs(out, exist_ok=True)
    recs = []
    for p in series:
        r = one(out, p, 75, True)
        recs.append(r)
        with open(os.path.join(out, "proxy_prof.json"), "w") as f:
            json.dump(recs, f, indent=1)
        print(json.dumps({k: r[k] for k in ("procs", "rc", "timed_out", "wall_s")}), flush=True)
        if r["timed_out"] or r["rc"] != 0:
            break  # nothing more on the GPU after a stall


if __name__ == "__main__":
    main()
