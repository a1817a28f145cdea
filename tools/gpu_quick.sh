# quick GPU check: parity tests, then the headline bench (no CPU leg, no
# sub-lines); stops at the first failure
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_quick.log 2>&1 &&
timeout -k 10 300 python -u bench.py --no-cpu --no-extra "$@" > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err
