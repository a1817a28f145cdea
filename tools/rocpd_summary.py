#!/usr/bin/env python3
"""Summarise rocprofv3 output databases (rocpd SQLite, ROCm 7.2 default) into
the text files committed under profiles/.

  python tools/rocpd_summary.py gpurun_out/prof_r01 profiles/r01_prof

reads <dir>/ktrace/*.db (--kernel-trace --stats run) and every other
<dir>/<pass>/*.db (--pmc passes) and writes <out>_ktrace_stats.csv and
<out>_pmc.csv. FETCH_SIZE is reported raw and corrected (x2 on gfx950 for
wide coalesced reads, MI355X_MICROARCH.md HBM section); SQ cycle counters are
quad-cycles.
"""

import csv
import glob
import os
import sqlite3
import sys


def one_db(d):
    dbs = sorted(glob.glob(os.path.join(d, "*.db")))
    if not dbs:
        raise SystemExit(f"no rocpd database under {d}")
    return sqlite3.connect(dbs[0])


def kernel_stats(d, out):
    c = one_db(d)
    rows = list(c.execute("select name, total_calls, total_duration, average, percentage from top_kernels"))
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "calls", "total_us", "avg_us", "percent"])
        for name, calls, tot, avg, pct in rows:
            short = name.split("(")[0] if name.startswith("hg::") else name[:80]
            w.writerow([short, calls, f"{tot:.3f}", f"{avg:.3f}", f"{pct:.2f}"])
    return rows


def pmc(dirs, out):
    rows = []
    for d in dirs:
        c = one_db(d)
        q = ("select kernel_name, counter_name, count(*), avg(value), min(value), max(value), "
             "avg(vgpr_count), avg(sgpr_count), avg(lds_block_size), avg(scratch_size) "
             "from counters_collection group by kernel_name, counter_name")
        for kn, cn, n, avg, lo, hi, vg, sg, lds, scr in c.execute(q):
            rows.append((os.path.basename(d), kn.split("(")[0], cn, n, avg, lo, hi, vg, sg, lds, scr))
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["pass", "kernel", "counter", "dispatches", "avg", "min", "max", "vgpr", "sgpr", "lds_bytes",
                    "scratch_bytes", "note"])
        for r in rows:
            note = ""
            if r[2] == "FETCH_SIZE":
                note = f"KB; x2 gfx950 correction = {2 * r[4] / 1024:.3f} MB per dispatch"
            elif r[2] == "WRITE_SIZE":
                note = f"KB = {r[4] / 1024:.3f} MB per dispatch"
            elif r[2].startswith("SQ_WAIT") or r[2] == "SQ_WAVE_CYCLES":
                note = "quad-cycles summed over waves"
            w.writerow(list(r[:4]) + [f"{r[4]:.1f}", f"{r[5]:.1f}", f"{r[6]:.1f}", int(r[7]), int(r[8]), int(r[9]),
                                      int(r[10]), note])
    return rows


def main():
    src, out = sys.argv[1], sys.argv[2]
    ks = kernel_stats(os.path.join(src, "ktrace"), out + "_ktrace_stats.csv")
    if os.path.isdir(os.path.join(src, "ktrace_all")):  # every sub-line of the bench, beside the headline alone
        kernel_stats(os.path.join(src, "ktrace_all"), out + "_ktrace_stats_all.csv")
    passes = [p for p in sorted(glob.glob(os.path.join(src, "*")))
              if os.path.isdir(p) and not os.path.basename(p).startswith("ktrace")]
    pm = pmc(passes, out + "_pmc.csv") if passes else []
    for r in ks[:3]:
        print(r[0].split("(")[0], r[1], f"avg {r[3]:.1f} us")
    for r in pm:
        print(r[0], r[2], f"{r[4]:.1f}")


if __name__ == "__main__":
    main()
