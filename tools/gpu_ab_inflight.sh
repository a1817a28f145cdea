#!/bin/bash
# Headline with 3..6 batches in flight (bench.py --inflight), interleaved
# three times on one box (--no-cpu --no-extra, 100 timed steps).
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r06if}
O=gpurun_out/ab_$T
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2 3; do
  for v in ${IF_VALUES:-3 4 5 6}; do
    timeout -k 10 240 python -u bench.py --steps 100 --warmup 20 --no-cpu --no-extra --inflight $v > $O/$v.$rep.json 2> $O/$v.$rep.err || exit $?
  done
done
python3 - $O <<'PY'
import json, sys, glob, os
o = sys.argv[1]
rows = {}
for f in sorted(glob.glob(os.path.join(o, "[0-9]*.json"))):
    v = os.path.basename(f).split(".")[0]
    d = json.loads(open(f).read().strip().splitlines()[-1])
    rows.setdefault(v, []).append((d["value"], d["ms_per_step"], d["hw_queues"]))
out = {v: {"value": [r[0] for r in rs], "ms_per_step": [r[1] for r in rs], "hw_queues": rs[0][2]} for v, rs in rows.items()}
json.dump(out, open(os.path.join(o, "summary.json"), "w"), indent=1)
print(json.dumps(out))
PY
