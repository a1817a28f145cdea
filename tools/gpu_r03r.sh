#!/bin/bash
# Full GPU suite + smoke + the default bench line, then a headline kernel
# timeline (rocprofv3 kernel trace summarised on the box).
set -o pipefail
cd $GRAFT_REPO_ROOT
R=${1:-r03r}
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu_$R.log 2>&1 &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$R.log 2>&1 &&
timeout -k 10 500 python -u bench.py > $O/bench_$R.json 2> $O/bench_$R.err &&
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tl_$R -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu --no-extra > $O/tl_$R.log 2>&1
rc=$?
if [ -d $O/tl_$R ]; then
  python3 tools/step_timeline.py $O/tl_$R > $O/tl_$R.txt 2>&1
  rm -f $O/tl_$R/*/*.db $O/tl_$R/*.db
fi
exit $rc
