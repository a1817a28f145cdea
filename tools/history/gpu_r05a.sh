#!/bin/bash
# r05: the headline-path oracle test first, the whole GPU suite, then the
# 2-rank gloo rehearsal started by bench.py itself (--gpus 2, no torchrun)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r05a}
timeout -k 10 300 python -u -m pytest tests/test_gpu_headline_path.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_${T}_head.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_${T}.log 2>&1 &&
HG_BENCH_BACKEND=gloo timeout -k 10 500 python -u bench.py --gpus 2 --no-cpu --steps 10 --warmup 3 > gpurun_out/bench_${T}_gloo2.json 2> gpurun_out/bench_${T}_gloo2.err
