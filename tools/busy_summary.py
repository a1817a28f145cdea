#!/usr/bin/env python3
"""Per-step device-busy time of the headline from a kernel trace of the
driver's invocation (rocprofv3 --kernel-trace, rocpd SQLite), so the line's
roofline fraction can be recomputed from a committed profile.

  python tools/busy_summary.py <trace dir> <bench line json> <out.json>

With batches in flight the kernels of several steps overlap (two pairing
launches share every SIMD), so a kernel's average launch duration says
nothing about a step. What a step costs the device is the UNION of all kernel
intervals inside the timed region, divided by the steps: bench.py records the
timed region on every host clock (`timed_region_ns`), this tool takes the
clock whose window holds the trace's kernels, clips every kernel interval to
the window and merges them. Writes {steps, busy_ms_per_step,
window_ms_per_step, idle_fraction, kernels, per_kernel}; bench.py's
`frac_rocprof` divides the step's implemented work by busy_ms_per_step.
"""

import glob
import json
import os
import sqlite3
import sys


def kernel_rows(d):
    """(name, start, end) of every dispatch in every rocpd database under d."""
    rows = []
    for db in sorted(glob.glob(os.path.join(d, "**", "*.db"), recursive=True)):
        c = sqlite3.connect(db)
        try:
            cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
            if not cols:
                continue
            name = "name" if "name" in cols else "kernel_name"
            rows += list(c.execute(f"select {name}, start, end from kernels"))
        finally:
            c.close()
    return rows


def union_ns(iv):
    total, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                total += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        total += cur_e - cur_s
    return total


def summarise(rows, marks, steps):
    best = None
    for clock, (t0, t1) in marks.items():
        inside = [(n, max(s, t0), min(e, t1)) for n, s, e in rows if e > t0 and s < t1]
        if best is None or len(inside) > len(best[1]):
            best = (clock, inside, t0, t1)
    clock, inside, t0, t1 = best
    if not inside:
        raise SystemExit("no kernel of the trace lies inside the timed region on any clock")
    busy = union_ns([(s, e) for _, s, e in inside])
    per = {}
    for n, s, e in inside:
        k = n.split("(")[0]
        d = per.setdefault(k, [0, 0.0])
        d[0] += 1
        d[1] += (e - s) / 1e3
    return {"clock": clock, "steps": steps, "kernels": len(inside),
            "window_ms_per_step": round((t1 - t0) / 1e6 / steps, 4),
            "busy_ms_per_step": round(busy / 1e6 / steps, 4),
            "idle_fraction": round(1 - busy / (t1 - t0), 4),
            "per_kernel": {k: {"dispatches_per_step": round(v[0] / steps, 2),
                               "kernel_us_per_step": round(v[1] / steps, 1)}
                           for k, v in sorted(per.items(), key=lambda kv: -kv[1][1])}}


def main():
    trace, line_path, out = sys.argv[1:4]
    with open(line_path) as f:
        line = json.loads([ln for ln in f.read().splitlines() if ln.startswith("{")][-1])
    marks = line.get("timed_region_ns")
    if not marks:
        raise SystemExit("the bench line has no timed_region_ns")
    res = summarise(kernel_rows(trace), marks, line["steps"])
    res["bench_ms_per_step"] = line["ms_per_step"]
    res["batches_in_flight"] = line.get("batches_in_flight")
    res["source"] = {"trace": trace, "line": line_path}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: res[k] for k in ("clock", "kernels", "busy_ms_per_step", "window_ms_per_step",
                                          "bench_ms_per_step")}))


if __name__ == "__main__":
    main()
