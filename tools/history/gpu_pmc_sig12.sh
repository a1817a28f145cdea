#!/bin/bash
# SQ counters of the two signature pairing kernels, one batch at a time
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r05f}
OUT=gpurun_out/pmc_$T
mkdir -p $OUT
export TMPDIR=/tmp
H="bench.py --no-cpu --no-extra --inflight 1 --steps 10 --warmup 2 --prewarm 0"
K="k_verify_sig|k_sig_"
HG_SIG12=1 timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY --kernel-include-regex "$K" -d $OUT/sq12 -o run -- python3 $H > $OUT/sq12.log 2>&1 &&
HG_SIG12=0 timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY --kernel-include-regex "$K" -d $OUT/sq16 -o run -- python3 $H > $OUT/sq16.log 2>&1 &&
HG_SIG12=1 timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_WAIT_INST_LDS --kernel-include-regex "$K" -d $OUT/mem12 -o run -- python3 $H > $OUT/mem12.log 2>&1 &&
HG_SIG12=0 timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_WAIT_INST_LDS --kernel-include-regex "$K" -d $OUT/mem16 -o run -- python3 $H > $OUT/mem16.log 2>&1 &&
mkdir -p $OUT/ktrace && python3 - <<PY
import glob, os, sqlite3
for d in sorted(glob.glob("$OUT/*/")):
    dbs = glob.glob(d + "*.db")
    if not dbs: continue
    c = sqlite3.connect(dbs[0])
    for kn, cn, n, avg in c.execute("select kernel_name, counter_name, count(*), avg(value) from counters_collection group by kernel_name, counter_name"):
        print(os.path.basename(d.rstrip('/')), kn.split('(')[0][:40], cn, n, round(avg, 1))
PY
