# Round 5: c4csg whole frames under other tile-order splits (RT_ORDER_TOP:
# the costliest 1/N of the tiles first, default 4); interleaved rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_order_ab}
mkdir -p $O
b() {  # name top config
  RT_ORDER_TOP=$2 timeout -k 10 300 python3 bench.py --config $3 --steps 20 --warmup 3 --cpu-baseline off --companion off > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/$1.json')); print('%-14s %.4f ms/step' % ('$1', d['ms_per_step']))"
}
for r in 1 2; do
  for t in ${TOPS:-4 2 3 6 1}; do b csg_top${t}_$r $t c4csg || exit 1; done
  for t in ${C3TOPS:-}; do b c3_top${t}_$r $t c3 || exit 1; done
done
