# Round-end rehearsal: full GPU tests, smoke(), default bench line, rocprofv3
# kernel stats, C3 PMC passes, sweep of every config (CPU baselines), brute-force band.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/r2}
mkdir -p $O/sweep
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail $O/bench_default.err; exit 1; }
cat $O/bench_default.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --cpu-baseline off > $O/bench_prof.json 2> $O/bench_prof.err || { tail $O/bench_prof.err; exit 1; }
find $O/prof -name '*kernel_stats.csv' | head -1 | xargs cat
bash scripts/gpu_pmc.sh c3 > $O/pmc_c3.log 2>&1 || { echo "pmc failed"; tail -20 $O/pmc_c3.log; exit 1; }
for c in c1 c2 canned c3 c3cone c4 c4csg c5; do
  steps=10; [ $c = c5 ] && steps=3; [ $c = c4csg ] && steps=5
  timeout -k 10 400 python bench.py --config $c --steps $steps --warmup 1 > $O/sweep/$c.json 2> $O/sweep/$c.err || { echo "sweep $c failed"; tail -5 $O/sweep/$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/sweep/$c.json')); print('$c', d['ms_per_step'], 'ms', d['value'], d['unit'], d['roofline']['frac'])"
done
timeout -k 10 400 python bench.py --config c5 --accel none --rows 2048:2304 --steps 1 --warmup 1 > $O/sweep/c5_bf_band.json 2> $O/sweep/c5_bf_band.err || { echo "brute failed"; tail -5 $O/sweep/c5_bf_band.err; exit 1; }
cat $O/sweep/c5_bf_band.json
