#!/bin/bash
# headline + sub-lines, no CPU leg
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --no-cpu > gpurun_out/bench_${1:-x}.json 2> gpurun_out/bench_${1:-x}.err
