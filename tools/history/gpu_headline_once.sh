#!/bin/bash
# the driver's default bench invocation once, plus the box's GPU identity (box-variance record)
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r05bx}
mkdir -p gpurun_out
(rocm-smi --showproductname --showclocks 2>/dev/null | head -40) > gpurun_out/${T}_smi.txt || true
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
