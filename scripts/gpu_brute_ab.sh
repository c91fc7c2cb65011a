# A/B of brute-force kernel variants (RT_SPEC_EXTRA_FLAGS) on a full-width C5
# row band.  usage: bash scripts/gpu_brute_ab.sh ROWS "FLAGS_A" "FLAGS_B" ...
# (an empty string = the default build)
set -o pipefail
cd $GRAFT_REPO_ROOT
ROWS=$1; shift
mkdir -p gpurun_out/ab
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -k "brute or stream" --timeout 300 --timeout-method thread > gpurun_out/pytest_brute.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_brute.log; exit 1; }
tail -1 gpurun_out/pytest_brute.log
n=0
for f in "$@"; do
  n=$((n+1))
  if [ -n "$f" ]; then export RT_SPEC_EXTRA_FLAGS="$f"; else unset RT_SPEC_EXTRA_FLAGS; fi
  timeout -k 10 400 python3 bench.py --config c5 --accel none --rows $ROWS --steps 1 --warmup 1 --cpu-baseline off > gpurun_out/ab/v$n.json 2> gpurun_out/ab/v$n.err || { echo "variant $n failed"; tail -5 gpurun_out/ab/v$n.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ab/v$n.json')); print('[$f]', d['ms_per_step'], 'ms', d['roofline']['frac'])"
done
