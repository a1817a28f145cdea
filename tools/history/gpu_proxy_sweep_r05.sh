#!/bin/bash
# config-4 proxy (service model) sweep on the final tree: lanes and fold overlap
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r05ps}
mkdir -p gpurun_out
P=handel_amd/_build/handel_proxy
L=handel_amd/_build/libhandel_gpu.so
: > gpurun_out/${T}.jsonl
CFGS=${CFGS:-"-l 8|-l 6|-l 12|-l 8 -o 0|-l 16"}
IFS='|' read -ra CS <<< "$CFGS"
for rep in 1 2 3 4; do
  for cfg in "${CS[@]}"; do
    out=$(env $ENVV timeout -k 10 120 $P $L -D 1 -P 1 $cfg 2> gpurun_out/${T}.err | tail -1) || exit 1
    echo "{\"cfg\": \"$cfg $ENVV\", \"rep\": $rep, \"r\": $out}" >> gpurun_out/${T}.jsonl
  done
done
