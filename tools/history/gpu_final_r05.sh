#!/bin/bash
# Round-5 record of the final tree: the GPU suite and smoke, config 5 on one
# GPU, the 2-rank rehearsal started by bench.py itself, then the driver's
# bench invocation pinned to its kernel trace and PMC passes (tools/gpu_pin.sh;
# last: runs after PMC passes measured config 5 at a half or a sixth of its
# rate, r05x / r05z)
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r05z}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_${T}.log 2>&1 &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${T}.log 2>&1 &&
timeout -k 10 300 python -u bench.py --committees --no-cpu --no-extra --steps 20 --warmup 5 > gpurun_out/bench_${T}_c5.json 2> gpurun_out/bench_${T}_c5.err &&
HG_BENCH_BACKEND=gloo timeout -k 10 500 python -u bench.py --gpus 2 --no-cpu --no-extra --steps 10 --warmup 3 > gpurun_out/bench_${T}_gloo2.json 2> gpurun_out/bench_${T}_gloo2.err &&
bash tools/gpu_pin.sh $T
