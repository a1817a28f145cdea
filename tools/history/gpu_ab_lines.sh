#!/bin/bash
# Normalised G2Base lines in k_verify_sig: GT-path parity tests, then an
# interleaved headline A/B against the HEAD library (variants/base)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_gt.py tests/test_gpu_gt_scope.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_lines.log 2>&1 || exit 1
echo "tests ok"
VARIANTS="base cur" bash tools/ab_variants.sh ${1:-r03z}
