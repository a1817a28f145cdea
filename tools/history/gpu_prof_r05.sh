#!/bin/bash
# kernel trace of the headline (default) and of the sequential line
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r05d}
OUT=gpurun_out/prof_$T
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/ktrace -o run -- python3 bench.py --no-cpu --no-extra --steps 20 --warmup 5 > $OUT/inflight.json 2> $OUT/inflight.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/ktrace_all -o run -- python3 bench.py --no-cpu --no-extra --inflight 1 --steps 20 --warmup 5 > $OUT/seq.json 2> $OUT/seq.err &&
python3 tools/rocpd_summary.py $OUT $OUT/${T} && rm -f $OUT/*/*.db
