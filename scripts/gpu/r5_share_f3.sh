# Round 5: C3 / C4 strong-scaling shares with 3 frames in flight vs 2
# (scripts/inflight_emul.py, every rank's share, slowest counts).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_share_f3}
mkdir -p $O
for r in 1 2; do
  for c in c3 c4; do
    INFLIGHT_F=2,3 INFLIGHT_WORLDS=1,4,8 timeout -k 10 400 python3 scripts/inflight_emul.py $c 20 > $O/${c}_$r.json 2> $O/${c}_$r.err || { tail -5 $O/${c}_$r.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/${c}_$r.json'))
for F in (2, 3):
    print('$c r$r F=%d' % F, '  '.join('w%d %.4f (%s)' % (w, d['w%d_f%d_max_ms' % (w, F)], d.get('w%d_f%d_eff_max' % (w, F))) for w in (1, 4, 8)))"
  done
done
