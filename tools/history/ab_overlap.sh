#!/bin/bash
# A/B of the fold beside the pairing kernel (HG_GT_OVERLAP=1, default) vs in sequence.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
B="bench.py --steps 30 --warmup 5 --no-cpu --pipeline 1"
for i in 1 2; do
timeout -k 10 300 env HG_GT_OVERLAP=0 python -u $B > gpurun_out/ab_${1}_seq_$i.json 2>/dev/null &&
timeout -k 10 300 env HG_GT_OVERLAP=1 python -u $B > gpurun_out/ab_${1}_ovl_$i.json 2>/dev/null || exit 1
done
