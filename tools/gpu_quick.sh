# quick GPU check: parity tests, then the bench (no CPU leg); stops at the first failure
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 200 python -u bench.py --no-cpu "$@" > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err
