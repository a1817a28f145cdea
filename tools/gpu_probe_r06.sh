#!/bin/bash
# Round 6 probes: the pairing kernels alone (tools/probe_sig12.py) with the
# product library and a probe variant (VARIANTS, handel_amd/_build/variants),
# interleaved, then one SQ pass per library on the 12-lane kernels.
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r06p}
O=gpurun_out/probe_$T
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  for v in cur ${VARIANTS:-noinv}; do
    lib=handel_amd/_build/variants/libhandel_gpu_$v.so
    [ $v = cur ] && lib=handel_amd/_build/libhandel_gpu.so
    HG_LIB=$lib timeout -k 10 120 python3 -u tools/probe_sig12.py > $O/$v.$rep.json 2> $O/$v.$rep.err || exit $?
  done
done
for v in cur ${VARIANTS:-noinv}; do
  lib=handel_amd/_build/variants/libhandel_gpu_$v.so
  [ $v = cur ] && lib=handel_amd/_build/libhandel_gpu.so
  HG_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_INSTS_SALU --kernel-include-regex "k_verify_sig12|k_sig_" -d $O/sq_$v -o run -- python3 tools/probe_sig12.py > $O/sq_$v.log 2>&1 || exit $?
done
python3 - $O <<'PY'
import sqlite3, glob, os, sys, json
o = sys.argv[1]
res = {}
for d in sorted(glob.glob(os.path.join(o, "sq_*"))):
    if not os.path.isdir(d):
        continue
    db = glob.glob(os.path.join(d, "**", "*.db"), recursive=True)[0]
    c = sqlite3.connect(db)
    q = "select kernel_name, counter_name, avg(value) from counters_collection group by kernel_name, counter_name"
    res[os.path.basename(d)] = {f"{k.split('(')[0]} {n}": v for k, n, v in c.execute(q)}
json.dump(res, open(os.path.join(o, "sq_summary.json"), "w"), indent=1)
for f in sorted(glob.glob(os.path.join(o, "*.json"))):
    print(os.path.basename(f), open(f).read().strip()[:600])
PY
