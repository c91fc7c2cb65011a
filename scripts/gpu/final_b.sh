# Round-5 evidence, part B: every config's bench line with its CPU baseline,
# and the GPU test suite.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/final_r5}
mkdir -p $O/sweep
for c in ${SWEEP_CFGS:-c1 c2 canned c3 c3cone c4 c4csg c5}; do
  steps=10; [ $c = c5 ] && steps=3; [ $c = c4csg ] && steps=20  # (c4csg: 20 frames, so the two-in-flight pipeline start does not dominate)
  timeout -k 10 400 python3 bench.py --config $c --steps $steps --warmup 1 --companion off > $O/sweep/$c.json 2> $O/sweep/$c.err || { echo "bench $c failed"; tail -5 $O/sweep/$c.err; exit 1; }
  echo "$c $(python3 -c "import json;d=json.load(open('$O/sweep/$c.json'));print(d['ms_per_step'], d['value'], d['roofline'].get('frac'), d['roofline'].get('executed_frac'))")"
done
timeout -k 10 700 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -1 $O/pytest_gpu.log; exit $rc
