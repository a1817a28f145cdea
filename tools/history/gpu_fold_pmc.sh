#!/bin/bash
# PMC passes of the GT fold alone on the full-registry batch
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r05fp}
OUT=gpurun_out/$T
mkdir -p $OUT
K="k_gt_chunks|k_gt_combine|k_gt_plan|k_verify_sig"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/ktrace -o run -- python3 tools/fold_pmc_driver.py > $OUT/kt.log 2>&1 &&
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY --kernel-include-regex "$K" -d $OUT/sq -o run -- python3 tools/fold_pmc_driver.py > $OUT/sq.log 2>&1 &&
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS --kernel-include-regex "$K" -d $OUT/mem -o run -- python3 tools/fold_pmc_driver.py > $OUT/mem.log 2>&1 &&
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$K" -d $OUT/fetch -o run -- python3 tools/fold_pmc_driver.py > $OUT/fetch.log 2>&1 &&
python3 tools/rocpd_summary.py $OUT $OUT/${T} && rm -f $OUT/*/*.db
