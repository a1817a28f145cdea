#!/bin/bash
# the GPU suite + smoke, then the bench with the 6-lane fold on and off (A/B).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 840 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_k6.log 2>&1 &&
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_k6.log 2>&1 &&
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu --no-service > gpurun_out/bench_k6.json 2> gpurun_out/bench_k6.err &&
HG_GT_K6=0 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu --no-service > gpurun_out/bench_k6off.json 2> gpurun_out/bench_k6off.err
