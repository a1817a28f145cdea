#!/bin/bash
# config 5 and the headline, no profiler anywhere in the call (box variance record)
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r05c5}
mkdir -p gpurun_out
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --committees --no-cpu --no-extra --steps 100 --warmup 20 > gpurun_out/${T}_c5_${rep}.json 2> gpurun_out/${T}_c5_${rep}.err &&
  timeout -k 10 300 python -u bench.py --no-cpu --no-extra --steps 100 --warmup 20 > gpurun_out/${T}_c3_${rep}.json 2> gpurun_out/${T}_c3_${rep}.err || exit 1
done
