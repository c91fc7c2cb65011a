# Quick check of HEAD: device exactness check, GPU parity suite, C3 counters + time.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 tests/hip/div_check 256 || exit 1
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 600 bash scripts/gpu_valu_ab.sh c3 "" "$@" || exit 1
timeout -k 10 600 bash scripts/gpu_tune.sh "c3 c2" "" "$@"
