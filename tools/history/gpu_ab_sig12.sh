#!/bin/bash
# A/B of the 12-lane signature pairing (HG_SIG12=1, the default) against the
# 16-lane k_verify_sig (HG_SIG12=0): parity first, then interleaved headline
# runs (four batches in flight) and the sequential / full-registry lines.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r05b}
timeout -k 10 300 python -u -m pytest tests/test_gpu_headline_path.py tests/test_gpu_gt.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_${T}_sig12.log 2>&1 || exit 1
for rep in 1 2; do
  for v in 1 0; do
    HG_SIG12=$v timeout -k 10 200 python -u bench.py --no-cpu --no-extra --steps 100 --warmup 20 > gpurun_out/ab_${T}_sig12_${v}_${rep}.json 2> gpurun_out/ab_${T}_sig12_${v}_${rep}.err || exit 1
  done
done
for v in 1 0; do
  HG_SIG12=$v timeout -k 10 200 python -u bench.py --no-cpu --inflight 1 --no-extra --steps 100 --warmup 20 > gpurun_out/ab_${T}_seq_${v}.json 2> gpurun_out/ab_${T}_seq_${v}.err || exit 1
done
