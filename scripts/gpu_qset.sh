# After the queue changes: full GPU tests, strong-scaling rehearsal, C3 bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/qset
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/qset/pytest.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/qset/pytest.log; exit 1; }
tail -1 gpurun_out/qset/pytest.log
for c in c3 c2 c4; do
  STRONG_WORLDS=1,2,4,8,270 timeout -k 10 300 python3 scripts/strong_emul.py $c > gpurun_out/qset/$c.json 2> gpurun_out/qset/$c.err || { echo "strong $c failed"; tail -5 gpurun_out/qset/$c.err; exit 1; }
  cat gpurun_out/qset/$c.json
done
for i in 1 2; do
  timeout -k 10 200 python3 bench.py --steps 30 --warmup 3 --cpu-baseline off > gpurun_out/qset/bench$i.json 2> gpurun_out/qset/bench$i.err || { tail -5 gpurun_out/qset/bench$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/qset/bench$i.json')); print('c3', d['ms_per_step'], d['roofline']['kernel_ms'])"
done
