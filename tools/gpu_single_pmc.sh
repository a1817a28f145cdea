#!/bin/bash
# HBM passes over config 2's k_verify (the `single` line's roofline traffic):
# FETCH_SIZE and WRITE_SIZE, one pass each -> gpurun_out/single_TAG/
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=${1:-r05s}
OUT=gpurun_out/single_$R
mkdir -p $OUT
S="bench.py --steps 5 --warmup 1 --no-cpu --no-service --pipeline 1"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_verify<" -d $OUT/fetch -o run -- python3 $S > $OUT/fetch.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_verify<" -d $OUT/write -o run -- python3 $S > $OUT/write.log 2>&1 &&
mkdir -p $OUT/ktrace && cp -r $OUT/fetch/* $OUT/ktrace/ 2>/dev/null; python3 - $OUT $OUT/${R} <<'PY'
import sys, os
sys.path.insert(0, "tools")
import rocpd_summary as R
src, out = sys.argv[1], sys.argv[2]
rows = R.pmc([os.path.join(src, "fetch"), os.path.join(src, "write")], out + "_single_pmc.csv")
for r in rows:
    print(r[0], r[1], r[2], f"{r[4]:.1f}")
PY
rm -f $OUT/*/*.db
