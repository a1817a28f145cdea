#!/bin/bash
# config-4 proxy sweep over the verifier service's lanes / queues / overlap / linger.
# usage: tools/gpu_proxy_sweep.sh TAG "name:args" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=$1; shift
P=handel_amd/_build/handel_proxy
L=handel_amd/_build/libhandel_gpu.so
for spec in "$@"; do
  n=${spec%%:*}; a=${spec#*:}
  timeout -k 10 120 $P $L -p 8 -k 250 -n 2000 -r 45 $a > gpurun_out/proxy_${tag}_${n}.json 2> gpurun_out/proxy_${tag}_${n}.err || exit 1
done
