#!/bin/bash
# kernel trace (rocpd database kept) of the headline one batch at a time
# (--inflight 1: the `sequential` form), for tools/step_timeline.py
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r05ts}
OUT=gpurun_out/trace_$T
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/kt -o run -- python3 bench.py --steps 40 --warmup 5 --no-cpu --no-extra --inflight 1 > $OUT/bench.json 2> $OUT/bench.err
