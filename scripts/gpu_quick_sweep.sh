# GPU-only timing of the configs (no CPU baseline): ms/frame per config.
# usage: bash scripts/gpu_quick_sweep.sh "c2 c3 c3cone c4 c4csg" [extra bench args]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/qsweep
mkdir -p $O
for c in ${1:-c2 c3 c3cone c4 c4csg}; do
  steps=20; [ $c = c5 ] && steps=3; [ $c = c4csg ] && steps=5
  timeout -k 10 300 python3 bench.py --config $c --steps $steps --warmup 2 --cpu-baseline off --companion off $2 > $O/$c.json 2> $O/$c.err || { echo "$c failed"; tail -3 $O/$c.err; exit 1; }
  echo "$c $(python3 -c "import json;d=json.load(open('$O/$c.json'));print(d['ms_per_step'], d['value'], d['roofline']['kernel_ms'])")"
done
