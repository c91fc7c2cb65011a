# Round 5: c4csg whole frames with 2 / 3 / 4 frames in flight, device board
# off and on (interleaved, two rounds).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_csg_inflight}
mkdir -p $O
b() {  # name config [extra bench args]
  n=$1; c=$2; shift 2
  timeout -k 10 300 python3 bench.py --config $c --steps 20 --warmup 3 --cpu-baseline off --companion off "$@" > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); print('%-16s %.4f ms/step  kernel %.4f' % ('$n', d['ms_per_step'], d['roofline']['kernel_ms']))"
}
for r in 1 2; do
  for f in 2 3 4; do
    b off_f$f.$r c4csg --inflight $f --work-sharing off && b dev_f$f.$r c4csg --inflight $f --work-sharing device || exit 1
  done
done
