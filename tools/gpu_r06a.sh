#!/bin/bash
# Round 6, first GPU session: the GPU suite (with the RCCL world-1 test) and
# smoke on the current tree, the driver's invocation pinned (gpu_pin.sh, now
# with the busy summary), and last the contexts-model proxy under rocprofv3
# with 1, 2, 8 processes (tools/proxy_prof.py stops at the first stall).
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r06a}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_${T}.log 2>&1 &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${T}.log 2>&1 &&
bash tools/gpu_pin.sh $T &&
timeout -k 10 400 python3 tools/proxy_prof.py gpurun_out/proxyprof_${T} 1 2 8 > gpurun_out/proxyprof_${T}.log 2>&1
