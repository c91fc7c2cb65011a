set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
RT_LDS_FULL=2 timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_full2.log 2>&1 || { echo "pytest full2 failed"; tail -30 gpurun_out/pytest_gpu_full2.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_full2.log
bash scripts/gpu_tune.sh "c3 c2" "" "RT_LDS_FULL=1|" "RT_LDS_FULL=1 RT_LDS_LEVELS=1|" "RT_LDS_LEVELS=1|"
