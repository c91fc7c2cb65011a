# Strong-scaling rehearsal on one GPU at the final build: every rank's share
# of a frame (interleaved 8-row tile rows) timed at 1/2/4/8 ranks, serial and
# with two frames in flight (scripts/inflight_emul.py).
# usage: bash scripts/gpu_r4_strong.sh TAG "CFGS" [FS]   (INFLIGHT_SHARE=1: work sharing)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-strong}; CFGS=${2:-"c2 c3 c3cone c4 c4csg c5"}
O=gpurun_out/r4_$TAG
mkdir -p $O
for c in $CFGS; do
  S=20; [ $c = c5 ] && S=3; [ $c = c4csg ] && S=10
  INFLIGHT_F=${3:-1,2} timeout -k 10 400 python3 scripts/inflight_emul.py $c $S > $O/inflight_$c.json 2> $O/inflight_$c.err || { tail -5 $O/inflight_$c.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/inflight_$c.json'))
print('$c', ' '.join('w%d: %.3f/%s' % (w, d['w%d_f2_max_ms' % w], d.get('w%d_f2_eff_max' % w)) for w in (1, 2, 4, 8)))"
done
