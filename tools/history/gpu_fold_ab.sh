#!/bin/bash
# fold A/B of a library variant against the in-tree library, interleaved:
# tools/fold_chunk_ab.py (headline and full registry: one batch at a time,
# four in flight, fold alone / beside the pairing)
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r05fa}
V=${2:-cw3}
mkdir -p gpurun_out
for rep in 1 2; do
  for v in cur $V; do
    lib=handel_amd/_build/variants/libhandel_gpu_$v.so
    [ $v = cur ] && lib=handel_amd/_build/libhandel_gpu.so
    HG_LIB=$lib timeout -k 10 300 python -u tools/fold_chunk_ab.py > gpurun_out/${T}_${v}_${rep}.json 2> gpurun_out/${T}_${v}_${rep}.err || exit 1
  done
done
