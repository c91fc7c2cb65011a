# GPU parity tests, then the brute-force search (bench --accel none: no BVH, no
# culling; BASELINE config 5's regime) beside the accelerated search.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/brute
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for spec in "c5 480 270 none" "c5 480 270 bvh" "c3 3840 2160 none"; do
  set -- $spec
  timeout -k 10 300 python bench.py --config $1 --width $2 --height $3 --accel $4 --steps 3 --warmup 1 --cpu-baseline auto > gpurun_out/brute/$1_$2_$4.json 2> gpurun_out/brute/$1_$2_$4.err || { echo "FAIL $spec"; tail -5 gpurun_out/brute/$1_$2_$4.err; exit 1; }
  cat gpurun_out/brute/$1_$2_$4.json
done
