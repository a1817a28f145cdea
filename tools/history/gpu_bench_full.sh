#!/bin/bash
# The driver's default bench line (headline, sub-lines, CPU baselines), then
# kernel-trace stats and the HBM-traffic PMC passes of the headline workload.
# Stops at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
R=${1:-r02}
OUT=gpurun_out/prof_$R
mkdir -p $OUT
export TMPDIR=/tmp
B="bench.py --steps 5 --warmup 2 --no-cpu --no-extra"
K="k_verify|k_gt_|k_agg_"
timeout -k 10 500 python -u bench.py > $OUT/bench_full.json 2> $OUT/bench_full.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/ktrace -o run -- python3 $B > $OUT/ktrace.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$K" -d $OUT/fetch -o run -- python3 $B > $OUT/fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$K" -d $OUT/write -o run -- python3 $B > $OUT/write.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY --kernel-include-regex "$K" -d $OUT/sq -o run -- python3 $B > $OUT/sq.log 2>&1
