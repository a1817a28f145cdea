#!/bin/bash
# GT-path tests + smoke, the bench with the 6-lane fold on / off and with two
# checks per pairing wave or without the one-wave-per-SIMD padding (A/B),
# then the whole GPU suite. A plain test failure of the GT tests (exit 1, not
# a crash or a time limit) is followed by the same tests on the 12-lane fold
# (HG_GT_K6=0), to tell the fold from the pairing kernel's layout.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
B="python3 bench.py --steps 20 --warmup 5 --no-cpu --no-service"
timeout -k 10 300 python -u -m pytest tests/test_gpu_gt.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gt.log 2>&1
rc=$?
if [ $rc -eq 1 ]; then
  HG_GT_K6=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_gt.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gt_k6off.log 2>&1
  exit 1
fi
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_k6.log 2>&1 &&
timeout -k 10 300 $B > gpurun_out/bench_k6.json 2> gpurun_out/bench_k6.err &&
HG_GT_K6=0 timeout -k 10 300 $B > gpurun_out/bench_k6off.json 2> gpurun_out/bench_k6off.err &&
HG_SIG_TEAMS=2 timeout -k 10 300 $B > gpurun_out/bench_t2.json 2> gpurun_out/bench_t2.err &&
HG_SIG_PAD=0 timeout -k 10 300 $B > gpurun_out/bench_pad0.json 2> gpurun_out/bench_pad0.err &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_all.log 2>&1
