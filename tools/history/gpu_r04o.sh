#!/bin/bash
# batches in flight on lanes (world 1: two queues per lane): 4, 5, 6, 4, 8
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
B="python3 bench.py --steps 20 --warmup 5 --no-cpu --no-service --no-extra"
timeout -k 10 300 $B --inflight 4 > gpurun_out/bench_r04o_4a.json 2> gpurun_out/bench_r04o_4a.err &&
timeout -k 10 300 $B --inflight 5 > gpurun_out/bench_r04o_5.json 2> gpurun_out/bench_r04o_5.err &&
timeout -k 10 300 $B --inflight 6 > gpurun_out/bench_r04o_6.json 2> gpurun_out/bench_r04o_6.err &&
timeout -k 10 300 $B --inflight 4 > gpurun_out/bench_r04o_4b.json 2> gpurun_out/bench_r04o_4b.err &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_gt.py -x -v -k lanes --timeout 120 --timeout-method thread > gpurun_out/pytest_r04o.log 2>&1
