#!/bin/bash
# r03q: packet-intake tests, the batcher and policy tests, the default bench
# (every sub-line, packet_intake included) and a headline kernel timeline.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u __graft_entry__.py smoke > $O/smoke_r03q.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_packets.py tests/test_gpu_gt.py tests/test_gpu_boundary.py tests/test_registry.py -m gpu -x -v \
  --timeout 300 --timeout-method thread -k "packet or crossing or batcher or registry" > $O/pytest_r03q.log 2>&1 &&
timeout -k 10 600 python bench.py > $O/bench_r03q.json 2> $O/bench_r03q.err &&
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tl_r03q -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu --no-extra > $O/tl_r03q.log 2>&1
rc=$?
python3 tools/step_timeline.py $O/tl_r03q/* > $O/tl_r03q.txt 2>&1
rm -f $O/tl_r03q/*/*.db $O/tl_r03q/*.db
exit $rc
