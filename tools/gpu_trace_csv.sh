#!/bin/bash
# kernel trace (rocpd database kept: per-dispatch start/end) of the headline
# bench, for a timeline of the lanes' kernels (tools/lane_timeline.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r05tl}
OUT=gpurun_out/trace_$T
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/kt -o run -- python3 bench.py --steps 30 --warmup 5 --no-cpu --no-extra > $OUT/bench.json 2> $OUT/bench.err
