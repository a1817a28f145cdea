#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ifs
for rep in 1 2; do
  for k in 3 4 5 6 8; do
    timeout -k 10 200 python -u bench.py --inflight $k --no-cpu --no-extra --steps 100 --warmup 20 > gpurun_out/ifs/k$k.$rep.json 2> gpurun_out/ifs/k$k.$rep.err || exit $?
  done
done
python3 - <<'PY'
import json,glob,os
rows={}
for f in sorted(glob.glob('gpurun_out/ifs/*.json')):
    k=os.path.basename(f).split('.')[0]
    d=json.loads(open(f).read().strip().splitlines()[-1]); rows.setdefault(k,[]).append(d['value'])
print(json.dumps(rows))
json.dump(rows, open('gpurun_out/ifs/summary.json','w'))
PY
