#!/bin/bash
# quick kernel-trace stats of the headline bench (one rocprofv3 pass)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=${1:-kt}
mkdir -p gpurun_out/$R
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$R/ktrace -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu --no-extra > gpurun_out/$R/ktrace.log 2>&1
