#!/bin/bash
# Variant A/B of the headline, then a kernel trace of the headline summarised
# per step (tools/step_timeline.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
export TMPDIR=/tmp
bash tools/ab_variants.sh r03s > $O/ab_r03s.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tl_r03s -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu --no-extra > $O/tl_r03s.log 2>&1
rc=$?
python3 tools/step_timeline.py $O/tl_r03s > $O/tl_r03s.txt 2>&1
find $O/tl_r03s -name '*.db' -delete
exit $rc
