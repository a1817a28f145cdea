#!/bin/bash
# New GPU tests (proxy), then the driver-default bench line, then a config-4 proxy run.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_proxy.py -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_proxy_${1:-t}.log 2>&1 &&
timeout -k 10 600 python -u bench.py > gpurun_out/bench_${1:-t}.json 2> gpurun_out/bench_${1:-t}.err &&
timeout -k 10 300 handel_amd/_build/handel_proxy handel_amd/_build/libhandel_gpu.so -p 8 -k 250 -n 2000 -r 45 -w 16 > gpurun_out/proxy_${1:-t}_policy.json 2> gpurun_out/proxy_${1:-t}_policy.err &&
timeout -k 10 300 handel_amd/_build/handel_proxy handel_amd/_build/libhandel_gpu.so -p 8 -k 250 -n 2000 -r 45 -w 16 -P 1 > gpurun_out/proxy_${1:-t}_prepared.json 2> gpurun_out/proxy_${1:-t}_prepared.err
