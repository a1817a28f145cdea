#!/bin/bash
# config-4 proxy (service model), interleaved runs over the values of one
# environment knob (default HG_SIG_W2_LANE_MAX: the two-wave pairing kernel on
# the service's lanes up to that many checks; HG_SERVICE_W2: the service's
# wave-budget policy for it)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r05sw}
REPS=${2:-2}
VALS=${3:-"0 512 1024 2048"}
VAR=${4:-HG_SIG_W2_LANE_MAX}
for rep in $(seq 1 $REPS); do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 200 python -c "import json, bench; print(json.dumps(bench.config4_proxy('service')))" > gpurun_out/${T}_${v}_${rep}.json 2> gpurun_out/${T}_${v}_${rep}.err || exit 1
  done
done
