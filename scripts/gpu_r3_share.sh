# Work sharing (RT_SHARE) check: full GPU parity suite, smoke, C3 bench,
# tail diagnostics and the strong-scaling rehearsal.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/r3share}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
timeout -k 10 300 python bench.py --cpu-baseline off > $O/bench_c3.json 2> $O/bench_c3.err || { tail $O/bench_c3.err; exit 1; }
cat $O/bench_c3.json
for c in c3 c4 c4csg; do
  RT_AMD_LIB=build_variants/librtamd_phase.so RT_SPEC_EXTRA_FLAGS="-DRT_PHASE_TIMING" timeout -k 10 200 python bench.py --config $c --steps 3 --warmup 1 --cpu-baseline off > $O/phase_$c.json 2> $O/phase_$c.err || { tail $O/phase_$c.err; exit 1; }
  echo "== $c $(python3 -c "import json; print(json.load(open('$O/phase_$c.json'))['ms_per_step'])")"; grep -E "waves|tail" $O/phase_$c.err | tail -2
done
for c in c4 c4csg c2; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --cpu-baseline off > $O/bench_$c.json 2> $O/bench_$c.err || { tail $O/bench_$c.err; exit 1; }
  echo "$c $(python3 -c "import json; print(json.load(open('$O/bench_$c.json'))['ms_per_step'])") ms"
done
for c in c3 c4; do
  timeout -k 10 300 python3 scripts/strong_emul.py $c > $O/strong_$c.json 2> $O/strong_$c.err || { tail -5 $O/strong_$c.err; exit 1; }
  cat $O/strong_$c.json
done
