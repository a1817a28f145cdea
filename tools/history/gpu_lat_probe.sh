#!/bin/bash
# latency timing probe of a (possibly wrong-valued) diagnostic variant against
# the in-tree library: tools/latency_ab.py --no-proxy kernel times only
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r05probe}
V=${2:-noredc}
mkdir -p gpurun_out
for rep in 1 2; do
  for v in cur $V; do
    lib=handel_amd/_build/variants/libhandel_gpu_$v.so
    [ $v = cur ] && lib=handel_amd/_build/libhandel_gpu.so
    HG_LIB=$lib timeout -k 10 200 python -u tools/latency_ab.py --no-proxy --no-check > gpurun_out/${T}_${v}_${rep}.json 2> gpurun_out/${T}_${v}_${rep}.err || exit 1
  done
done
