# Bench A/B of kernel variants over several configs (no tests).
# usage: bash scripts/gpu_modes.sh "CONFIGS" "FLAGS_A" "FLAGS_B" ...   ("" = default)
set -o pipefail
cd $GRAFT_REPO_ROOT
CFGS=$1; shift
mkdir -p gpurun_out/modes
for c in $CFGS; do
  for f in "$@"; do
    if [ -n "$f" ]; then export RT_SPEC_EXTRA_FLAGS="$f"; else unset RT_SPEC_EXTRA_FLAGS; fi
    extra=""; steps=10
    case $c in c5bf) cfg=c5; extra="--accel none --rows 2048:2304"; steps=1;; c5) cfg=c5; steps=3;; *) cfg=$c;; esac
    timeout -k 10 300 python3 bench.py --config $cfg $extra --steps $steps --warmup 1 --cpu-baseline off > "gpurun_out/modes/$c$f.json" 2> "gpurun_out/modes/$c$f.err" || { echo "bench $c $f failed"; tail -5 "gpurun_out/modes/$c$f.err"; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/modes/$c$f.json')); print('$c [$f]', d['ms_per_step'], 'ms')"
  done
done
