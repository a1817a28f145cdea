#!/bin/bash
# latency A/B of a library variant against the in-tree library, interleaved
# (tools/latency_ab.py --no-proxy), plus the cross-kernel FE test on the variant
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r05lv}
V=${2:-rp}
mkdir -p gpurun_out
HG_LIB=handel_amd/_build/variants/libhandel_gpu_$V.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_headline_path.py -k identical_fe > gpurun_out/${T}_fe.log 2>&1 || exit 1
for rep in 1 2 3; do
  for v in cur $V; do
    lib=handel_amd/_build/variants/libhandel_gpu_$v.so
    [ $v = cur ] && lib=handel_amd/_build/libhandel_gpu.so
    HG_LIB=$lib timeout -k 10 200 python -u tools/latency_ab.py --no-proxy > gpurun_out/${T}_${v}_${rep}.json 2> gpurun_out/${T}_${v}_${rep}.err || exit 1
  done
done
