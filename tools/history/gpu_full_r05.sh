#!/bin/bash
# the whole GPU suite, smoke, then the driver's bench invocation (all lines)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r05g}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_${T}.log 2>&1 &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${T}.log 2>&1 &&
timeout -k 10 900 python -u bench.py > gpurun_out/bench_${T}.json 2> gpurun_out/bench_${T}.err
