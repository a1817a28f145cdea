#!/bin/bash
# The bench line pinned to a profile of the same invocation:
#  1. the driver's invocation, plain (bench.json);
#  2. the same invocation under --kernel-trace --stats: its bench line and its
#     per-kernel averages come from ONE run (bench_traced.json, *_driver_ktrace_stats.csv);
#     and the per-step device-busy time of its timed region (tools/busy_summary.py:
#     the union of the kernel intervals inside it / steps -> *_driver_busy.json);
#  3. PMC passes of the headline alone (HBM bytes, SQ counters), one counter
#     group per run, and one HBM pass over the config-2 `single` line's
#     k_verify and the stream's k_verify_ml (their rooflines' traffic).
# usage: tools/gpu_pin.sh TAG   -> gpurun_out/pin_TAG/
set -o pipefail
cd $GRAFT_REPO_ROOT
R=${1:-r05}
OUT=gpurun_out/pin_$R
mkdir -p $OUT
export TMPDIR=/tmp
D="bench.py --steps 20 --warmup 5"
H="bench.py --steps 20 --warmup 5 --no-cpu --no-extra"
S="bench.py --steps 5 --warmup 1 --no-cpu --no-service --pipeline 1"
K="k_verify_sig|k_sig_|k_sig12|k_gt_|k_agg_"
timeout -k 10 600 python3 $D > $OUT/bench.json 2> $OUT/bench.err &&
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $OUT/ktrace -o run -- python3 $D > $OUT/bench_traced.json 2> $OUT/traced.err &&
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$K" -d $OUT/fetch -o run -- python3 $H > $OUT/fetch.log 2>&1 &&
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$K" -d $OUT/write -o run -- python3 $H > $OUT/write.log 2>&1 &&
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY --kernel-include-regex "$K" -d $OUT/sq -o run -- python3 $H > $OUT/sq.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_verify<|k_verify_ml" -d $OUT/single_fetch -o run -- python3 $S > $OUT/single_fetch.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_verify<|k_verify_ml" -d $OUT/single_write -o run -- python3 $S > $OUT/single_write.log 2>&1 &&
python3 tools/rocpd_summary.py $OUT $OUT/${R}_driver &&
python3 tools/busy_summary.py $OUT/ktrace $OUT/bench_traced.json $OUT/${R}_driver_busy.json && rm -f $OUT/*/*.db
