# Per-config timing (frames in flight 2 and serial), no CPU baseline.
# usage: bash scripts/gpu_r4_sweep.sh TAG "CFGS" [extra bench args]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-sweep}; CFGS=${2:-"c3 c4 c5"}; shift 2
O=gpurun_out/r4_$TAG
mkdir -p $O
for c in $CFGS; do
  S=20; [ $c = c5 ] && S=4; [ $c = c4csg ] && S=10
  timeout -k 10 300 python3 bench.py --config $c --steps $S --warmup 2 --cpu-baseline off --companion off "$@" > $O/f2_$c.json 2> $O/f2_$c.err || { tail -5 $O/f2_$c.err; exit 1; }
  timeout -k 10 300 python3 bench.py --config $c --steps $S --warmup 2 --inflight 1 --cpu-baseline off --companion off "$@" > $O/f1_$c.json 2> $O/f1_$c.err || { tail -5 $O/f1_$c.err; exit 1; }
  python3 -c "import json; a=json.load(open('$O/f2_$c.json')); b=json.load(open('$O/f1_$c.json')); print('$c inflight2 %.4f ms/step (kernel %.4f)  serial %.4f ms' % (a['ms_per_step'], a['roofline']['kernel_ms'], b['roofline']['kernel_ms']))"
done
