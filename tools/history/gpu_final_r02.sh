#!/bin/bash
# Closing check of a round-2 tree on one GPU box: the GPU parity suite, smoke,
# the driver-default bench line (CPU legs included), then kernel-trace stats
# and separate PMC passes (HBM traffic, SQ counters) of the bench with its
# sub-lines, so k_verify (config 2), k_verify_sig and the fold are all covered.
# Stops at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
R=${1:-r02}
OUT=gpurun_out/prof_$R
mkdir -p $OUT
export TMPDIR=/tmp
B="bench.py --steps 5 --warmup 2 --no-cpu --pipeline 1"
K="k_verify|k_gt_|k_agg_"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$R.log 2>&1 &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$R.log 2>&1 &&
timeout -k 10 500 python -u bench.py > $OUT/bench_full.json 2> $OUT/bench_full.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/ktrace -o run -- python3 $B > $OUT/ktrace.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$K" -d $OUT/fetch -o run -- python3 $B > $OUT/fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$K" -d $OUT/write -o run -- python3 $B > $OUT/write.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY --kernel-include-regex "$K" -d $OUT/sq -o run -- python3 $B > $OUT/sq.log 2>&1
