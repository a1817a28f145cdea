#!/bin/bash
# batches in flight on lanes: 3 (twice), 4, 3 padded, 2
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
B="python3 bench.py --steps 20 --warmup 5 --no-cpu --no-service --no-extra"
timeout -k 10 300 $B --inflight 3 > gpurun_out/bench_r04l_3a.json 2> gpurun_out/bench_r04l_3a.err &&
timeout -k 10 300 $B --inflight 4 > gpurun_out/bench_r04l_4.json 2> gpurun_out/bench_r04l_4.err &&
HG_SIG_PAD=1 timeout -k 10 300 $B --inflight 3 > gpurun_out/bench_r04l_3pad.json 2> gpurun_out/bench_r04l_3pad.err &&
timeout -k 10 300 $B --inflight 2 > gpurun_out/bench_r04l_2.json 2> gpurun_out/bench_r04l_2.err &&
timeout -k 10 300 $B --inflight 3 > gpurun_out/bench_r04l_3b.json 2> gpurun_out/bench_r04l_3b.err &&
timeout -k 10 300 $B --inflight 1 > gpurun_out/bench_r04l_1.json 2> gpurun_out/bench_r04l_1.err
