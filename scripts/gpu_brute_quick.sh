# Brute-force parity tests (streamed / scalar-load paths vs the oracle), then
# the C5 full-width band PMC script.  usage: bash scripts/gpu_brute_quick.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -k "brute or stream" --timeout 300 --timeout-method thread > gpurun_out/pytest_brute.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_brute.log; exit 1; }
tail -2 gpurun_out/pytest_brute.log
bash scripts/gpu_brute_pmc.sh ${1:-smem}
