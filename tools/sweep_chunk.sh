#!/bin/bash
# fold schedule sweep (HG_GT_CHUNK x HG_GT_GRID) on the headline and full-registry batches
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sweep
for cfg in ${SWEEP:-"8 4096" "12 4096" "16 4096" "24 4096" "32 4096" "16 8192"}; do
  set -- $cfg
  HG_GT_CHUNK=$1 HG_GT_GRID=$2 timeout -k 10 200 python3 tools/fold_probe.py > gpurun_out/sweep/c$1_g$2.json 2>/dev/null || exit 1
done
