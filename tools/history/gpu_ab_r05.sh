#!/bin/bash
# interleaved headline A/B on one box: the default kernel choice and HG_SIG12=0
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r05q}
for rep in 1 2 3; do
  for v in auto 0; do
    if [ $v = auto ]; then E=""; else E="HG_SIG12=$v"; fi
    env $E timeout -k 10 200 python -u bench.py --no-cpu --no-extra --steps 100 --warmup 20 > gpurun_out/ab_${T}_${v}_${rep}.json 2> gpurun_out/ab_${T}_${v}_${rep}.err || exit 1
  done
done
timeout -k 10 300 python -u bench.py --committees --no-cpu --no-extra --steps 20 --warmup 5 > gpurun_out/ab_${T}_c5.json 2> gpurun_out/ab_${T}_c5.err
