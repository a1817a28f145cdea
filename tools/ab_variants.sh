#!/bin/bash
# Headline A/B of library variants (handel_amd/_build/variants/*.so, built
# from earlier commits) against the in-tree library, interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
R=${1:-r03s}
O=gpurun_out/ab_$R
mkdir -p $O
V=handel_amd/_build/variants
for rep in 1 2 3; do
  for v in ${VARIANTS:-lazy lazyef cur}; do
    lib=$V/libhandel_gpu_$v.so
    [ $v = cur ] && lib=handel_amd/_build/libhandel_gpu.so
    HG_LIB=$lib timeout -k 10 240 python -u bench.py --steps ${AB_STEPS:-100} --warmup 20 ${AB_FLAGS:---no-cpu --no-extra} > $O/$v.$rep.json 2> $O/$v.$rep.err || exit $?
    echo "$v $rep done"
  done
done
python3 - $O <<'PY'
import json, sys, glob, os
rows = {}
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.json"))):
    v = os.path.basename(f).split(".")[0]
    d = json.loads(open(f).read().strip().splitlines()[-1])
    fr = d.get("full_registry", {}).get("value")
    rows.setdefault(v, []).append((d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"], d["roofline_k_verify"]["kernel_ms"], d["roofline_gt_fold"]["kernel_ms"], fr))
out = {v: {"value": [r[0] for r in rs], "ms_per_step": [r[1] for r in rs], "submit_ms": [r[2] for r in rs], "k_verify_sig_alone_ms": [r[3] for r in rs], "fold_alone_ms": [r[4] for r in rs], "full_registry": [r[5] for r in rs]} for v, rs in rows.items()}
json.dump(out, open(os.path.join(sys.argv[1], "summary.json"), "w"), indent=1)
print(json.dumps(out))
PY
