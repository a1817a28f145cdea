#!/bin/bash
# GPU suite, then the config-4 proxy in both process models (r04: the verifier service).
# usage: tools/gpu_service.sh TAG [tests|notests]
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-t}
P=handel_amd/_build/handel_proxy
L=handel_amd/_build/libhandel_gpu.so
if [ "${2:-tests}" = tests ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_${tag}.log 2>&1 || exit 1
fi
run() {  # name, proxy args
  local n=$1; shift
  timeout -k 10 120 $P $L -p 8 -k 250 -n 2000 -r 45 "$@" > gpurun_out/proxy_${tag}_${n}.json 2> gpurun_out/proxy_${tag}_${n}.err
}
run daemon_l8 -D 1 -P 1 -l 8 &&
run daemon_l16_q16 -D 1 -P 1 -l 16 -Q 16 &&
run daemon_l8_q8_seq -D 1 -P 1 -l 8 -Q 8 -o 0 &&
run daemon_l16_q16_seq -D 1 -P 1 -l 16 -Q 16 -o 0 &&
run daemon_l32_q32_seq -D 1 -P 1 -l 32 -Q 32 -o 0 -u 20 &&
run contexts_prepared -D 0 -P 1 -w 16 &&
run daemon_policy -D 1 -P 0 -l 16 -Q 16
