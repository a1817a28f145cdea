#!/bin/bash
# kernel + memory-copy trace of the config-4 proxy (service model): where a
# service batch's wall time goes (tools/service_timeline.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r05tp}
OUT=gpurun_out/trace_$T
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/kt -o run -- handel_amd/_build/handel_proxy handel_amd/_build/libhandel_gpu.so -D 1 -P 1 -l 8 > $OUT/proxy.json 2> $OUT/proxy.err
