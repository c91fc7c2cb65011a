# Parity tests matching a -k filter, then bench A/B of kernel variants
# (RT_SPEC_EXTRA_FLAGS; "" = default) on one config.
# usage: bash scripts/gpu_cfg_ab.sh CONFIG "PYTEST_K" STEPS "FLAGS_A" "FLAGS_B" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
CFG=$1; K=$2; STEPS=$3; shift 3
mkdir -p gpurun_out/cab
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "$K" --timeout 300 --timeout-method thread > gpurun_out/pytest_cab.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_cab.log; exit 1; }
  tail -1 gpurun_out/pytest_cab.log
fi
n=0
for f in "$@"; do
  n=$((n+1))
  if [ -n "$f" ]; then export RT_SPEC_EXTRA_FLAGS="$f"; else unset RT_SPEC_EXTRA_FLAGS; fi
  timeout -k 10 400 python3 bench.py --config $CFG --steps $STEPS --warmup 1 --cpu-baseline off > gpurun_out/cab/v$n.json 2> gpurun_out/cab/v$n.err || { echo "variant $n failed"; tail -5 gpurun_out/cab/v$n.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/cab/v$n.json')); print('[$f]', d['ms_per_step'], 'ms', d['roofline']['frac'])"
done
