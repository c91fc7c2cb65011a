# Full GPU tests, then C3/C2/C4 with several RT_TAIL_WAVES (tail quarter tiles).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tail
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for c in c3 c2 c3cone; do
  for tw in 0 1 2 4; do
    RT_TAIL_WAVES=$tw timeout -k 10 300 python3 bench.py --config $c --steps 10 --warmup 2 --cpu-baseline off > gpurun_out/tail/$c-$tw.json 2> gpurun_out/tail/$c-$tw.err || { echo "bench failed"; tail -3 gpurun_out/tail/$c-$tw.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/tail/$c-$tw.json')); print('$c tail_waves=$tw', d['ms_per_step'], 'ms')"
  done
done
