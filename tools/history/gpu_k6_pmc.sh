#!/bin/bash
# SQ counters of the GT fold kernels alone, 6-lane vs 12-lane (tools/fold_probe.py),
# and the service tests.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/k6pmc; export TMPDIR=/tmp
K="k_gt_chunks|k_gt_combine|k_gt_win16"
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY"
timeout -k 10 300 python -u -m pytest tests/test_gpu_service.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_service.log 2>&1 &&
timeout -k 10 120 python3 tools/fold_probe.py > gpurun_out/k6pmc/probe_k6.json 2>&1 &&
HG_GT_K6=0 timeout -k 10 120 python3 tools/fold_probe.py > gpurun_out/k6pmc/probe_k6off.json 2>&1 &&
timeout -s KILL 180 rocprofv3 --pmc $C --kernel-include-regex "$K" -d gpurun_out/k6pmc/on -o run -- python3 tools/fold_probe.py > gpurun_out/k6pmc/on.log 2>&1 &&
HG_GT_K6=0 timeout -s KILL 180 rocprofv3 --pmc $C --kernel-include-regex "$K" -d gpurun_out/k6pmc/off -o run -- python3 tools/fold_probe.py > gpurun_out/k6pmc/off.log 2>&1
