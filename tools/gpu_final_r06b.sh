#!/bin/bash
# The round-6 record in two calls (each under gpurun's 20-minute limit):
#   part 1: the GPU suite and smoke, config 5, the 2-rank rehearsal (gloo);
#   part 2: the driver's invocation pinned (tools/gpu_pin.sh) and the
#           contexts-model proxy under rocprofv3 (tools/proxy_prof.py).
# usage: tools/gpu_final_r06b.sh TAG 1|2
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r06f}
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${2:-1}" = 1 ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_${T}.log 2>&1 &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${T}.log 2>&1 &&
timeout -k 10 300 python -u bench.py --committees --no-cpu --no-extra --steps 20 --warmup 5 > gpurun_out/bench_${T}_c5.json 2> gpurun_out/bench_${T}_c5.err &&
HG_BENCH_BACKEND=gloo timeout -k 10 500 python -u bench.py --gpus 2 --no-extra --steps 10 --warmup 3 --cpu-sample 512 > gpurun_out/bench_${T}_gloo2.json 2> gpurun_out/bench_${T}_gloo2.err
else
bash tools/gpu_pin.sh $T &&
timeout -k 10 400 python3 tools/proxy_prof.py gpurun_out/proxyprof_${T} 1 2 8 > gpurun_out/proxyprof_${T}.log 2>&1
fi
