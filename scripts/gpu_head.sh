# HEAD check: GPU test suite, smoke, default bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/head}
mkdir -p $O
timeout -k 10 700 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -1 $O/pytest_gpu.log; [ $rc = 0 ] || exit $rc
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
cat $O/bench_default.json
for c in ${INFLIGHT_CFGS:-c3 c4 c2}; do
  INFLIGHT_F=1,2,3 timeout -k 10 300 python3 scripts/inflight_emul.py $c 30 > $O/inflight_$c.json 2> $O/inflight_$c.err || { tail -5 $O/inflight_$c.err; exit 1; }
  cat $O/inflight_$c.json
done
