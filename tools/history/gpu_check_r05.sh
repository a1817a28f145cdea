#!/bin/bash
# quick check of a tree: the headline-path and GT parity tests, two headline
# bench runs and the latency helper (no proxy)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r05c}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_headline_path.py tests/test_gpu_gt.py > gpurun_out/${T}_pytest.log 2>&1 &&
timeout -k 10 200 python -u bench.py --no-cpu --no-extra --steps 100 --warmup 20 > gpurun_out/${T}_b1.json 2> gpurun_out/${T}_b1.err &&
timeout -k 10 200 python -u tools/latency_ab.py --no-proxy > gpurun_out/${T}_lat.json 2> gpurun_out/${T}_lat.err &&
timeout -k 10 200 python -u bench.py --no-cpu --no-extra --steps 100 --warmup 20 > gpurun_out/${T}_b2.json 2> gpurun_out/${T}_b2.err
