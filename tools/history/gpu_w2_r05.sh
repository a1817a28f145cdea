#!/bin/bash
# the two-wave latency kernel: parity (cross-kernel FE values, the headline
# path's verdicts, the GT path's runs), then an interleaved latency A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r05w}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_headline_path.py tests/test_gpu_gt.py > gpurun_out/${T}_pytest.log 2>&1 &&
for rep in 1 2; do
  for v in 1 0; do
    HG_SIG_W2=$v timeout -k 10 300 python -u tools/latency_ab.py > gpurun_out/${T}_lat_${v}_${rep}.json 2> gpurun_out/${T}_lat_${v}_${rep}.err || exit 1
  done
done
