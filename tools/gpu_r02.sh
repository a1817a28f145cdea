#!/bin/bash
# Round-2 GPU check: parity suite, smoke, then the full bench line (CPU legs
# included). Each GPU step has its own limit; the chain stops at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 400 python -u bench.py "$@" > gpurun_out/bench.json 2> gpurun_out/bench.err
