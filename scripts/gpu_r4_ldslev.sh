# Frame-core LDS levels (RT_LDS_LEVELS) vs whole frames and 8-rank shares
# (two frames in flight): fewer levels leave room for a fourth workgroup per
# CU when a workgroup's waves finish apart.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4_${1:-ldslev}
mkdir -p $O
for c in ${2:-c3 c4csg}; do for n in 9 2 1 0; do
  RT_LDS_LEVELS=$n INFLIGHT_WORLDS=1,8 INFLIGHT_F=2 timeout -k 10 300 python3 scripts/inflight_emul.py $c 12 > $O/${c}_l$n.json 2> $O/${c}_l$n.err || { tail -5 $O/${c}_l$n.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/${c}_l$n.json')); print('$c levels<=$n', d['w1_f2_max_ms'], d['w8_f2_max_ms'], d.get('w8_f2_eff_max'))"
done; done
