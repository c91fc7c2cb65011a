# rt_set_frames_in_flight: schedule-hint parity, and the strong/in-flight table with the hint.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/hint}
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_schedule.py tests/test_gpu_dist.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc = 0 ] || exit $rc
for c in c4 c3 c2 c4csg; do
  INFLIGHT_F=1,2,3 timeout -k 10 300 python3 scripts/inflight_emul.py $c 20 > $O/inflight_$c.json 2> $O/inflight_$c.err || { tail -5 $O/inflight_$c.err; exit 1; }
  echo $c; cat $O/inflight_$c.err | grep -v Warn
done
for c in c4 c5; do
  timeout -k 10 300 python3 bench.py --config $c --cpu-baseline off --steps 10 > $O/bench_$c.json 2> $O/bench_$c.err || { tail -5 $O/bench_$c.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$c.json'));r=d['roofline'];print('$c', d['ms_per_step'], d['value'], r['kernel_ms'], r['launch_ms_overlapped'])"
done
