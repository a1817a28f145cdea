#!/bin/bash
# Driver-default bench line (CPU legs included) of the current tree.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py > gpurun_out/bench_${1:-t}.json 2> gpurun_out/bench_${1:-t}.err
