#!/bin/bash
# Config 2's split form (launch_verify_split): parity of the config-2 GPU tests
# with it forced on, then one batch at a time and K in flight, split off / on.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/single_split_${1:-t}
mkdir -p $O
export TMPDIR=/tmp
HG_VERIFY_SPLIT=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
  -k "verify_batch or ragged or empty or hash_reject or pack_verdicts" > $O/pytest_split.log 2>&1 &&
for rep in 1 2; do
  for sp in 0 1; do
    HG_VERIFY_SPLIT=$sp timeout -k 10 200 python -u tools/single_inflight.py $O/split$sp.$rep.json 1 2 4 > $O/split$sp.$rep.log 2>&1 || exit $?
  done
done
