#!/bin/bash
# Headline A/B of one environment switch, interleaved on one box:
#   AB_VAR=HG_SIG12_SPLIT AB_VALUES="1 0" tools/gpu_ab_env.sh TAG
# (bench.py --no-cpu --no-extra, 100 timed steps, three rounds), then the
# pairing kernels alone (tools/probe_sig12.py) per value.
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r06ab}
O=gpurun_out/ab_$T
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2 3; do
  for v in ${AB_VALUES:-1 0}; do
    env $AB_VAR=$v timeout -k 10 240 python -u bench.py --steps ${AB_STEPS:-100} --warmup 20 ${AB_FLAGS:---no-cpu --no-extra} > $O/$v.$rep.json 2> $O/$v.$rep.err || exit $?
  done
done
for v in ${AB_VALUES:-1 0}; do
  env $AB_VAR=$v timeout -k 10 120 python3 -u tools/probe_sig12.py > $O/probe_$v.json 2> $O/probe_$v.err || exit $?
done
python3 - $O <<'PY'
import json, sys, glob, os
o = sys.argv[1]
rows = {}
for f in sorted(glob.glob(os.path.join(o, "[0-9]*.json"))):
    v = os.path.basename(f).split(".")[0]
    d = json.loads(open(f).read().strip().splitlines()[-1])
    rows.setdefault(v, []).append((d["value"], d["ms_per_step"], d["roofline"]["frac"],
                                   d.get("roofline_k_verify_sig12", {}).get("kernel_ms")))
out = {v: {"value": [r[0] for r in rs], "ms_per_step": [r[1] for r in rs], "frac": [r[2] for r in rs],
           "sig12_alone_ms": [r[3] for r in rs]} for v, rs in rows.items()}
for v in out:
    p = os.path.join(o, f"probe_{v}.json")
    if os.path.exists(p):
        out[v]["probe"] = json.loads(open(p).read().strip().splitlines()[-1])
json.dump(out, open(os.path.join(o, "summary.json"), "w"), indent=1)
print(json.dumps(out))
PY
