#!/bin/bash
# Config-4 proxy through the verifier service (handel_proxy -D 1 -P 1 -l 8):
# padded service lanes (16-lane pairing kernel, one wave per SIMD; default)
# vs unpadded ones (the 12-lane split pairing), interleaved three times.
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r06sp}
O=gpurun_out/svc_$T
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2 3; do
  for v in ${SP_VALUES:-1 0}; do
    HG_SERVICE_PAD=$v timeout -k 10 120 handel_amd/_build/handel_proxy handel_amd/_build/libhandel_gpu.so -D 1 -P 1 -l ${SP_LANES:-8} > $O/pad$v.$rep.json 2> $O/pad$v.$rep.err || exit $?
  done
done
python3 - $O <<'PY'
import json, sys, glob, os
o = sys.argv[1]
rows = {}
for f in sorted(glob.glob(os.path.join(o, "pad*.json"))):
    v = os.path.basename(f).split(".")[0]
    d = json.loads(open(f).read().strip().splitlines()[-1])
    rows.setdefault(v, []).append({"throughput": d["throughput"], "p50": d["latency_us"]["p50"],
                                   "p99": d["latency_us"]["p99"], "batches": d["batches"], "mismatches": d["mismatches"]})
json.dump(rows, open(os.path.join(o, "summary.json"), "w"), indent=1)
print(json.dumps(rows))
PY
