# C5 (BVH, global scene) with and without the tile-cost order (RT_TILE_ORDER=2
# extends it to BVH scenes outside LDS), serial and two frames in flight.
# usage: bash scripts/gpu_r4_c5order.sh TAG [CFG]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; CFG=${2:-c5}
O=gpurun_out/r4_$TAG
mkdir -p $O
for o in 1 2; do
  for f in 1 2; do
    RT_TILE_ORDER=$o timeout -k 10 300 python3 bench.py --config $CFG --steps 4 --warmup 1 --inflight $f --cpu-baseline off --companion off > $O/o${o}_f$f.json 2> $O/o${o}_f$f.err || { tail -5 $O/o${o}_f$f.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/o${o}_f$f.json')); print('order=$o F=$f', d['ms_per_step'], d['config'].get('tile_order_ms'))"
  done
done
