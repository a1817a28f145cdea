#!/bin/bash
# config 5 on one GPU, then 2-rank rehearsals of the multi-GPU bench (gloo
# collectives, both ranks on the one GPU of the box): headline and committees
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
R=${1:-r03}
timeout -k 10 300 python -u bench.py --committees --no-cpu --no-extra --steps 10 > gpurun_out/bench_${R}_c5.json 2> gpurun_out/bench_${R}_c5.err &&
HG_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --no-cpu --no-extra --steps 10 > gpurun_out/bench_${R}_gloo2.json 2> gpurun_out/bench_${R}_gloo2.err &&
HG_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --committees --no-cpu --no-extra --steps 10 > gpurun_out/bench_${R}_c5_gloo2.json 2> gpurun_out/bench_${R}_c5_gloo2.err
