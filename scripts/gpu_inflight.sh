# Frames in flight: GPU tests of the multi-context path, bench lines at F = 1 / 2 / 3,
# and a rocprofv3 kernel trace of the default bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/inflight}
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_dist.py -x -v --timeout 120 --timeout-method thread > $O/pytest_dist.log 2>&1; rc=$?; tail -3 $O/pytest_dist.log; [ $rc = 0 ] || exit $rc
for f in 2 1 3; do
  timeout -k 10 300 python3 bench.py --inflight $f --cpu-baseline off > $O/bench_c3_f$f.json 2> $O/bench_c3_f$f.err || { tail -5 $O/bench_c3_f$f.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_c3_f$f.json'));r=d['roofline'];print('c3 F=$f', d['ms_per_step'], d['value'], r['kernel_ms'], r['launch_ms_overlapped'], r['frac'], d['c3cone']['ms_per_step'])"
done
for c in c4 c2 c4csg; do
  for f in 2 1; do
    timeout -k 10 300 python3 bench.py --config $c --inflight $f --cpu-baseline off --steps 20 > $O/bench_${c}_f$f.json 2> $O/bench_${c}_f$f.err || { tail -5 $O/bench_${c}_f$f.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/bench_${c}_f$f.json'));r=d['roofline'];print('$c F=$f', d['ms_per_step'], d['value'], r['kernel_ms'], r['launch_ms_overlapped'])"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o c3 -- python3 bench.py --companion off --cpu-baseline off > $O/bench_c3_prof.json 2> $O/prof.err || { tail -5 $O/prof.err; exit 1; }
cat $O/bench_c3_prof.json
find $O/prof -name '*.csv' | head
