#!/bin/bash
# the fused-bitset test, then the lazy / lazy+EF / current A/B and the step probe
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_gt.py -m gpu -x -v -k fused --timeout 200 --timeout-method thread > $O/pytest_fused_r03u.log 2>&1 &&
bash tools/ab_variants.sh r03u > $O/ab_r03u.log 2>&1 &&
timeout -k 10 300 python -u tools/step_probe.py 40 > $O/step_probe_r03u.json 2> $O/step_probe_r03u.err
