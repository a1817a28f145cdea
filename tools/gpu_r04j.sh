#!/bin/bash
# the headline's two-lanes mode with hardware queues for every stream (bench
# default), padded vs unpadded, 4 queues, three lanes.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
B="python3 bench.py --steps 20 --warmup 5 --no-cpu --no-service"
timeout -k 10 300 $B > gpurun_out/bench_r04k_lanes.json 2> gpurun_out/bench_r04k_lanes.err &&
HG_SIG_PAD=1 timeout -k 10 300 $B --no-extra > gpurun_out/bench_r04k_lanes_pad.json 2> gpurun_out/bench_r04k_lanes_pad.err &&
HG_BENCH_HW_QUEUES=4 timeout -k 10 300 $B --no-extra > gpurun_out/bench_r04k_lanes_q4.json 2> gpurun_out/bench_r04k_lanes_q4.err &&
timeout -k 10 300 $B --inflight 3 --no-extra > gpurun_out/bench_r04k_lanes3.json 2> gpurun_out/bench_r04k_lanes3.err
