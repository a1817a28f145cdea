#!/usr/bin/env python3
"""Per-step timeline of the headline from a rocprofv3 --kernel-trace database
(rocpd SQLite): where the wall time of one bench step goes between two
consecutive pairing-kernel launches.

  python tools/step_timeline.py gpurun_out/prof_x/ktrace [anchor-regex]

For every anchor dispatch (default k_verify_sig<4, true>) after the first few,
lists the dispatches up to the next anchor with their start offset from the
anchor's start and their duration, then the mean period and the mean idle
time of the main stream (no kernel of the step running).
"""

import glob
import os
import re
import sqlite3
import statistics
import sys


def dispatches(d):
    db = sorted(glob.glob(os.path.join(d, "*.db")))[0]
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "name" if "name" in cols else "kernel_name"
    q = f"select {name}, start, end{', stream_id' if 'stream_id' in cols else ''} from kernels order by start"
    return cols, [r for r in c.execute(q)]


def main():
    d = sys.argv[1]
    anchor = re.compile(sys.argv[2] if len(sys.argv) > 2 else r"k_verify_sig<4, true(, (true|false))?>")
    cols, rows = dispatches(d)
    print("columns:", ",".join(cols))
    idx = [i for i, r in enumerate(rows) if anchor.search(r[0])]
    if len(idx) < 4:
        raise SystemExit(f"{len(idx)} anchor dispatches")
    periods, idle, busy_runs = [], [], {}
    for a, b in zip(idx[2:-1], idx[3:]):
        t0 = rows[a][1]
        periods.append((rows[b][1] - t0) / 1e3)
        # main-stream idle: the union of kernel intervals in [t0, next anchor)
        iv = sorted((r[1], r[2]) for r in rows[a:b])
        cover, cur_s, cur_e = 0, None, None
        for s, e in iv:
            e = min(e, rows[b][1])
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    cover += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        cover += cur_e - cur_s
        idle.append((rows[b][1] - t0 - cover) / 1e3)
        for r in rows[a:b]:
            k = r[0].split("(")[0][:60]
            busy_runs.setdefault(k, []).append(((r[1] - t0) / 1e3, (r[2] - r[1]) / 1e3))
    print(f"steps: {len(periods)}  period mean {statistics.mean(periods):.1f} us "
          f"(min {min(periods):.1f}, max {max(periods):.1f})  idle (no kernel) mean {statistics.mean(idle):.1f} us")
    for k, v in sorted(busy_runs.items(), key=lambda kv: statistics.mean(x[0] for x in kv[1])):
        print(f"  {k:60s} n/step {len(v) / len(periods):.2f}  start +{statistics.mean(x[0] for x in v):8.1f} us"
              f"  dur {statistics.mean(x[1] for x in v):8.1f} us")


if __name__ == "__main__":
    main()
