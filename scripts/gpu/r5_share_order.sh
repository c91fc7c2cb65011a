# Round 5: tile-order split (RT_ORDER_TOP) on C3's and c4's strong-scaling
# shares (4 and 8 ranks, two frames in flight); interleaved rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_share_order}
mkdir -p $O
run() {  # name top config
  RT_ORDER_TOP=$2 INFLIGHT_F=2 INFLIGHT_WORLDS=4,8 timeout -k 10 300 python3 scripts/inflight_emul.py $3 20 > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; return 1; }
  python3 -c "
import json; d=json.load(open('$O/$1.json'))
print('%-14s' % '$1', '  '.join('w%d %.4f (%s)' % (w, d['w%d_f2_max_ms' % w], d.get('w%d_f2_eff_max' % w)) for w in (4, 8)))"
}
for r in 1 2; do for t in 6 1 2 3 12; do run c3_t${t}_$r $t c3 || exit 1; done; done
