#!/bin/bash
# Diagnostic: k_verify time vs checks per wave (HG_TEAMS_PER_BLOCK = 4, 2, 1).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for t in 4 2 1; do
  HG_TEAMS_PER_BLOCK=$t timeout -k 10 200 python3 bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/tpb_$t.json 2>gpurun_out/tpb_$t.err || exit 1
done
