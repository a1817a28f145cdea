#!/bin/bash
# batches in flight sweep of the headline (12-lane pairing kernel)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r05r}
for rep in 1 2; do
  for k in 3 4 5 6; do
    timeout -k 10 200 python -u bench.py --no-cpu --no-extra --inflight $k --steps 100 --warmup 20 > gpurun_out/inf_${T}_${k}_${rep}.json 2> gpurun_out/inf_${T}_${k}_${rep}.err || exit 1
  done
done
