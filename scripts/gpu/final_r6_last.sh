# Round 6, last evidence pass at the final tree: part A (PMC for every config,
# the default bench line, rocprofv3 summary + spans, smoke), then the full GPU
# suite once.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/final_r6}
bash scripts/gpu/final_a.sh || exit 1
timeout -k 10 900 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -1 $O/pytest_gpu.log; exit $rc
