# Concurrent tail kernel (RT_TAIL_SPLIT): parity suite with a split, then C3/C2/c3cone timings per split.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/split
RT_TAIL_SPLIT=0.2 timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_split.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_split.log; exit 1; }
tail -1 gpurun_out/pytest_split.log
for c in c3 c2 c3cone; do
  for f in 0 0.05 0.1 0.2 0.3; do
    RT_TAIL_SPLIT=$f timeout -k 10 300 python3 bench.py --config $c --steps 10 --warmup 2 --cpu-baseline off > gpurun_out/split/$c-$f.json 2> gpurun_out/split/$c-$f.err || { echo "bench failed"; tail -3 gpurun_out/split/$c-$f.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/split/$c-$f.json')); print('$c split=$f', d['ms_per_step'], 'ms')"
  done
done
