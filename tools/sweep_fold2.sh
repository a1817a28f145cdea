#!/bin/bash
# headline (100 steps) over fold schedules (HG_GT_CHUNK x HG_GT_GRID), two passes
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/sweep_${1:-x}
mkdir -p $O
B="bench.py --steps 100 --warmup 20 --no-cpu --no-extra"
for rep in 1 2; do
for cfg in ${SWEEP:-"8 4096" "8 1024" "8 2048" "16 1024" "4 4096" "12 2048"}; do
  set -- $cfg
  HG_GT_CHUNK=$1 HG_GT_GRID=$2 timeout -k 10 200 python3 $B > $O/c$1_g$2.$rep.json 2>/dev/null || exit 1
  echo "$cfg $rep: $(python3 -c "import json;d=json.loads(open('$O/c$1_g$2.$rep.json').read().strip().splitlines()[-1]);r=d['roofline'];print(d['ms_per_step'], r['kernels_ms'])")"
done
done
