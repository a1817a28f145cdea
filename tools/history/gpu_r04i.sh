#!/bin/bash
# GT tests (incl. the device lanes), the bench with two batches in flight on
# lanes (default) and one at a time, then the service's linger sweep with the
# follow policy.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
B="python3 bench.py --steps 20 --warmup 5 --no-cpu --no-service"
timeout -k 10 300 python -u -m pytest tests/test_gpu_gt.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_r04i_gt.log 2>&1 &&
timeout -k 10 300 $B > gpurun_out/bench_r04i_lanes.json 2> gpurun_out/bench_r04i_lanes.err &&
timeout -k 10 300 $B --inflight 1 > gpurun_out/bench_r04i_seq.json 2> gpurun_out/bench_r04i_seq.err &&
timeout -k 10 300 $B > gpurun_out/bench_r04i_lanes2.json 2> gpurun_out/bench_r04i_lanes2.err &&
bash tools/gpu_proxy_sweep.sh r04h "u100a:-D 1 -P 1 -l 8 -w 4 -u 100" "u50a:-D 1 -P 1 -l 8 -w 4 -u 50" "u200a:-D 1 -P 1 -l 8 -w 4 -u 200" "u100b:-D 1 -P 1 -l 8 -w 4 -u 100" "u50b:-D 1 -P 1 -l 8 -w 4 -u 50" "u200b:-D 1 -P 1 -l 8 -w 4 -u 200" "l10u100:-D 1 -P 1 -l 10 -w 4 -u 100" "l6u100:-D 1 -P 1 -l 6 -w 4 -u 100"
