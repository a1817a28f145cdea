#!/bin/bash
# lazy / lazy+EF / current A/B (three interleaved reps) and the step probe.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
export TMPDIR=/tmp
bash tools/ab_variants.sh r03t > $O/ab_r03t.log 2>&1 &&
timeout -k 10 300 python -u tools/step_probe.py 40 > $O/step_probe_r03t.json 2> $O/step_probe_r03t.err
