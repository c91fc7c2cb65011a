# Frames in flight x pixel schedule on the deep-glass configs (whole frames and 8-rank shares).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/inflight_sched}
mkdir -p $O
for c in c4 c4csg c3; do
  for q in 0 1; do
    RT_PIXEL_QUADS=$q INFLIGHT_WORLDS=${WORLDS:-1,8} INFLIGHT_F=1,2,3 timeout -k 10 300 python3 scripts/inflight_emul.py $c 20 > $O/${c}_q$q.json 2> $O/${c}_q$q.err || { tail -5 $O/${c}_q$q.err; exit 1; }
    echo "$c quads=$q"; cat $O/${c}_q$q.json
  done
done
