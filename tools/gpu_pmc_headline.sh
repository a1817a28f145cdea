#!/bin/bash
# PMC passes of the headline alone (one counter group per run): HBM bytes and
# the SQ instruction / cycle counters of every step kernel -> <TAG>_pmc.csv
set -o pipefail
cd $GRAFT_REPO_ROOT
R=${1:-r06d}
OUT=gpurun_out/pmc_$R
mkdir -p $OUT
export TMPDIR=/tmp
H="bench.py --steps 20 --warmup 5 --no-cpu --no-extra"
K="k_verify_sig|k_sig_|k_sig12|k_gt_|k_agg_"
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$K" -d $OUT/fetch -o run -- python3 $H > $OUT/fetch.log 2>&1 &&
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$K" -d $OUT/write -o run -- python3 $H > $OUT/write.log 2>&1 &&
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY --kernel-include-regex "$K" -d $OUT/sq -o run -- python3 $H > $OUT/sq.log 2>&1 &&
python3 - $OUT $R <<'PY'
import sys, os, importlib.util
spec = importlib.util.spec_from_file_location("rs", "tools/rocpd_summary.py")
rs = importlib.util.module_from_spec(spec); spec.loader.exec_module(rs)
out, r = sys.argv[1], sys.argv[2]
passes = [os.path.join(out, p) for p in ("fetch", "write", "sq")]
rs.pmc(passes, os.path.join(out, f"{r}_pmc.csv"))
PY
rm -f $OUT/*/*.db
