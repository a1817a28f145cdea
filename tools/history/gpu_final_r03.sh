#!/bin/bash
# Final-tree evidence: GPU suite, smoke, the driver-default bench line, then
# kernel-trace stats and PMC passes (tools/gpu_prof_r03.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
R=${1:-r03f}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$R.log 2>&1 &&
echo "tests ok" &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$R.log 2>&1 &&
echo "smoke ok" &&
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$R.json 2> gpurun_out/bench_$R.err &&
echo "bench ok" &&
bash tools/gpu_prof_r03.sh $R
