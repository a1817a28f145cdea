#!/bin/bash
# config-4 proxy (service model) with the two-wave pairing kernel allowed on
# the service's lanes for batches up to HG_SIG_W2_LANE_MAX checks, interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r05sw}
for rep in 1 2; do
  for v in 0 512 1024 2048; do
    HG_SIG_W2_LANE_MAX=$v timeout -k 10 200 python -c "import json, bench; print(json.dumps(bench.config4_proxy('service')))" > gpurun_out/${T}_${v}_${rep}.json 2> gpurun_out/${T}_${v}_${rep}.err || exit 1
  done
done
