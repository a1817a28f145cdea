# diagnostic: in-kernel phase timers (diag build) for both pairing-check
# kernels, then I-cache / issue counters of the two-wave kernel
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2d
export TMPDIR=/tmp
B="bench.py --steps 5 --warmup 2 --no-cpu --no-extra"
P="SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY"
timeout -k 10 200 python3 tools/diag.py > gpurun_out/r2d/diag2.json 2> gpurun_out/r2d/diag2.err &&
HG_VERIFY_1WAVE=1 timeout -k 10 200 python3 tools/diag.py > gpurun_out/r2d/diag1.json 2> gpurun_out/r2d/diag1.err &&
timeout -k 10 300 rocprofv3 --pmc $P --kernel-include-regex "k_verify" -d gpurun_out/r2d/ic2 -o run -- python3 $B > gpurun_out/r2d/ic2.log 2>&1 &&
HG_VERIFY_1WAVE=1 timeout -k 10 300 rocprofv3 --pmc $P --kernel-include-regex "k_verify" -d gpurun_out/r2d/ic1 -o run -- python3 $B > gpurun_out/r2d/ic1.log 2>&1
