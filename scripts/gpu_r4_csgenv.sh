# c4csg under LDS-budget experiments (same box, one ab.py process per setting):
# the scene in LDS or global, frame fields of the first levels in LDS.
# usage: bash scripts/gpu_r4_csgenv.sh TAG lib1 lib2 ...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/r4_$TAG
mkdir -p $O
i=0
for e in "RT_X=0" "RT_LDS_FULL=2" "RT_SCENE_GLOBAL=1" "RT_SCENE_GLOBAL=1 RT_LDS_FULL=3"; do
  i=$((i+1))
  env $e RT_DEBUG_LAUNCH=1 timeout -k 10 300 python3 scripts/ab.py --config c4csg --rounds 3 "$@" > $O/env$i.log 2> $O/env$i.err || { tail -5 $O/env$i.err; exit 1; }
  echo "== $e"; grep "^\[launch\]" $O/env$i.err | sort | uniq -c | head -4; grep '"lib"' $O/env$i.log
done
