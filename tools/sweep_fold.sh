#!/bin/bash
# GT-path tests, then the headline over fold schedules (HG_GT_CHUNK x HG_GT_GRID)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sweep
[ -n "$SKIP_TESTS" ] || timeout -k 10 500 python -u -m pytest tests/test_gpu_gt.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/sweep/pytest.log 2>&1 || exit 1
B="bench.py --steps 20 --warmup 3 --no-cpu --no-extra"
for cfg in ${SWEEP:-"8 4096" "8 8192" "8 16384" "10 8192" "6 8192" "12 16384"}; do
  set -- $cfg
  HG_GT_CHUNK=$1 HG_GT_GRID=$2 timeout -k 10 200 python3 $B > gpurun_out/sweep/c$1_g$2.json 2>/dev/null || exit 1
done
