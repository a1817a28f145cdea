#!/bin/bash
# full-registry in-flight sweep (tools/full_inflight_ab.py), default kernels and HG_SIG12=0
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r05fi}
timeout -k 10 400 python -u tools/full_inflight_ab.py > gpurun_out/${T}_auto.json 2> gpurun_out/${T}_auto.err &&
HG_SIG12=0 timeout -k 10 400 python -u tools/full_inflight_ab.py > gpurun_out/${T}_16.json 2> gpurun_out/${T}_16.err
