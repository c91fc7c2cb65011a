# Round 6: c4csg whole frames under each pixel schedule and frames in flight
# (bench.py --schedule / --inflight; the working tree's library), two rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/r6_csg_sched}
mkdir -p $O
for r in 1 2; do
  for s in quads pairs pixel; do
    for f in 2 3; do
      n=c4csg_${s}_f${f}_$r
      timeout -k 10 300 python3 bench.py --config c4csg --schedule $s --inflight $f --steps 20 --warmup 3 --cpu-baseline off --companion off > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/$n.json')); print('%-22s %.4f ms/step' % ('$n', d['ms_per_step']))"
    done
  done
done
