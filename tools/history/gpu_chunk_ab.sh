#!/bin/bash
# GT fold chunk-size A/B (tools/fold_chunk_ab.py), interleaved twice
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r05k}
for rep in 1 2; do
  for c in 8 16 32; do
    HG_GT_CHUNK=$c timeout -k 10 200 python -u tools/fold_chunk_ab.py >> gpurun_out/chunk_${T}.jsonl 2>> gpurun_out/chunk_${T}.err || exit 1
  done
done
