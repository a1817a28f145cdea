#!/bin/bash
# Round-2 profile on the GPU box (headline config-3 workload): kernel-trace
# stats of bench.py, then separate PMC passes (HBM traffic, then SQ
# instruction/stall counters) for the pairing check and the Combine fold.
# Each GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
R=${1:-r02}
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_$R
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
B="bench.py --steps 5 --warmup 2 --no-cpu --no-extra"
K="k_verify|k_aggregate|k_agg_|k_gt_"
timeout -k 10 300 python3 $B > $OUT/bench.json 2> $OUT/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/ktrace -o run -- python3 $B > $OUT/ktrace.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$K" -d $OUT/fetch -o run -- python3 $B > $OUT/fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$K" -d $OUT/write -o run -- python3 $B > $OUT/write.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY --kernel-include-regex "$K" -d $OUT/sq -o run -- python3 $B > $OUT/sq.log 2>&1
