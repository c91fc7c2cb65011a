# Specialised-kernel check: GPU parity tests, then benches with and without specialisation.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
for cfg in c4csg c3; do
  st=20; [ $cfg = c5 ] && st=3
  for sp in on off; do
    timeout -k 10 300 python bench.py --config $cfg --steps $st --warmup 2 --cpu-baseline off --specialize $sp > gpurun_out/bench_${cfg}_$sp.json 2> gpurun_out/bench_${cfg}_$sp.err || exit 1
  done
done
