#!/bin/bash
# Kernel-trace stats of the whole bench (every sub-line) and of the headline
# alone, then separate PMC passes (HBM traffic, SQ counters) of the headline
# alone, so per-dispatch averages are the headline batch's.
set -o pipefail
cd $GRAFT_REPO_ROOT
R=${1:-r03}
OUT=gpurun_out/prof_$R
mkdir -p $OUT
export TMPDIR=/tmp
B="bench.py --steps 5 --warmup 2 --no-cpu --pipeline 1"
H="bench.py --steps 10 --warmup 2 --no-cpu --no-extra"
K="k_verify|k_gt_|k_agg_"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/ktrace_all -o run -- python3 $B > $OUT/ktrace_all.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/ktrace -o run -- python3 $H > $OUT/ktrace.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$K" -d $OUT/fetch -o run -- python3 $H > $OUT/fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$K" -d $OUT/write -o run -- python3 $H > $OUT/write.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY --kernel-include-regex "$K" -d $OUT/sq -o run -- python3 $H > $OUT/sq.log 2>&1 &&
# summaries on the box; the rocpd databases stay there (gpurun_out returns <= 64 MiB)
python3 tools/rocpd_summary.py $OUT $OUT/$R && rm -f $OUT/*/*.db
