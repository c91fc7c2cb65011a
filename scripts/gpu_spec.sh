# Specialised-kernel check: GPU parity tests, then C3/C2 bench with and without specialisation.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
for cfg in c3 c2; do
  for sp in on off; do
    timeout -k 10 300 python bench.py --config $cfg --steps 20 --warmup 3 --cpu-baseline off --specialize $sp > gpurun_out/bench_${cfg}_$sp.json 2> gpurun_out/bench_${cfg}_$sp.err || exit 1
  done
done
RT_SPEC_EXTRA_FLAGS=-DRT_MIN_WAVES=4 timeout -k 10 300 python bench.py --config c3 --steps 20 --warmup 3 --cpu-baseline off > gpurun_out/bench_c3_w4.json 2> gpurun_out/bench_c3_w4.err || exit 1
