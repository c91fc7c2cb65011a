# Full GPU parity suite, then bench lines + wave-lifetime diagnostics for
# c3 / c4 / c4csg; extra args: RT_SPEC_EXTRA_FLAGS variants ("" = default).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/slots
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
fi
[ $# -eq 0 ] && set -- ""
for c in c3 c4 c4csg; do
  for f in "$@"; do
    if [ -n "$f" ]; then export RT_SPEC_EXTRA_FLAGS="$f"; else unset RT_SPEC_EXTRA_FLAGS; fi
    timeout -k 10 300 python3 bench.py --config $c --steps 10 --warmup 2 --cpu-baseline off > "gpurun_out/slots/$c$f.json" 2> "gpurun_out/slots/$c$f.err" || { echo "bench $c $f failed"; tail -5 "gpurun_out/slots/$c$f.err"; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/slots/$c$f.json')); print('$c [$f]', d['ms_per_step'], 'ms')"
  done
  unset RT_SPEC_EXTRA_FLAGS
  bash scripts/gpu_phase.sh $c || exit 1
done
