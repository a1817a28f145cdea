#!/bin/bash
# Instruction-fetch counters of the headline (is the 480 KB pairing kernel
# I-cache bound?): the available counter list, then small PMC passes
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/icache_${1:-x}
mkdir -p $O
export TMPDIR=/tmp
H="bench.py --steps 10 --warmup 2 --no-cpu --no-extra"
K="k_verify|k_gt_chunks"
timeout -s KILL 60 rocprofv3 --list-avail > $O/avail.txt 2>&1 || true
grep -o "SQC_[A-Z_]*\|SQ_IFETCH[A-Z_]*\|SQ_INSTS_[A-Z_]*\|SQ_WAIT_[A-Z_]*" $O/avail.txt | sort -u > $O/names.txt || true
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES --kernel-include-regex "$K" -d $O/ic1 -o run -- python3 $H > $O/ic1.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU --kernel-include-regex "$K" -d $O/ic2 -o run -- python3 $H > $O/ic2.log 2>&1
rc=$?
python3 tools/rocpd_summary.py $O $O/summary > $O/summary.log 2>&1 || true
du -sh $O/* > $O/sizes.txt 2>&1 || true
exit $rc
