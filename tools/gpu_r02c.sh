#!/bin/bash
# Round-2 A/B check of the tree: GPU parity suite, smoke, the bench line with
# its sub-lines (no CPU leg), then kernel-trace stats and one SQ counter pass
# of the headline. Stops at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
R=${1:-r02}
OUT=gpurun_out/prof_$R
mkdir -p $OUT
export TMPDIR=/tmp
B="bench.py --steps 5 --warmup 2 --no-cpu --no-extra"
K="k_verify|k_gt_"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$R.log 2>&1 &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$R.log 2>&1 &&
timeout -k 10 400 python -u bench.py --no-cpu > $OUT/bench_extra.json 2> $OUT/bench_extra.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/ktrace -o run -- python3 $B > $OUT/ktrace.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY --kernel-include-regex "$K" -d $OUT/sq -o run -- python3 $B > $OUT/sq.log 2>&1
