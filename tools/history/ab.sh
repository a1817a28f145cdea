# A/B timing of two builds on one box: $1 = env for A, $2 = env for B (each
# "VAR=value ..." or "-"); parity tests first, then headline bench lines
# alternated A B A B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
B="bench.py --steps 20 --warmup 3 --no-cpu --no-extra"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab/pytest.log 2>&1 || exit 1
for i in 1 2; do
  env ${1/#-/} timeout -k 10 200 python3 $B > gpurun_out/ab/a$i.json 2>/dev/null &&
  env ${2/#-/} timeout -k 10 200 python3 $B > gpurun_out/ab/b$i.json 2>/dev/null || exit 1
done
