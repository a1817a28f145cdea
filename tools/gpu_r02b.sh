#!/bin/bash
# Round-2 check of the tree: GPU parity suite, smoke, then the profile script
# (bench line, kernel-trace stats, PMC passes). Stops at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${1:-r02}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$R.log 2>&1 &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$R.log 2>&1 &&
bash tools/profile_r02.sh $R
