#!/bin/bash
# GPU suite + smoke + the driver-default bench line (CPU legs included).
set -o pipefail
cd $GRAFT_REPO_ROOT
R=${1:-r03}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$R.log 2>&1 &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$R.log 2>&1 &&
timeout -k 10 500 python -u bench.py > gpurun_out/bench_$R.json 2> gpurun_out/bench_$R.err
