# Round 5: the device-wide board on C3's strong-scaling shares (INFLIGHT_SHARE
# 2) vs off, two frames in flight, 1 / 4 / 8 ranks; interleaved rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_c3_share}
mkdir -p $O
run() {  # name share config
  INFLIGHT_SHARE=$2 INFLIGHT_F=2 INFLIGHT_WORLDS=1,4,8 timeout -k 10 300 python3 scripts/inflight_emul.py $3 20 > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; return 1; }
  python3 -c "
import json; d=json.load(open('$O/$1.json'))
print('%-14s' % '$1', '  '.join('w%d %.3f (%s)' % (w, d['w%d_f2_max_ms' % w], d.get('w%d_f2_eff_max' % w)) for w in (1, 4, 8)))"
}
for r in 1 2; do run c3_off$r 0 c3 && run c3_dev$r 2 c3 && run c2_off$r 0 c2 && run c2_dev$r 2 c2 || exit 1; done
