# Round 5: c4csg whole frame (two in flight) and 8-rank shares under
# kernel variants (hipRTC defines) and the global-scene flavour.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_csg_ab}
mkdir -p $O
run() {  # name extra-defines [env...]
  n=$1; f=$2; shift 2
  env "$@" RT_SPEC_EXTRA_FLAGS="$f" INFLIGHT_F=2 INFLIGHT_WORLDS=1,8 timeout -k 10 300 python3 scripts/inflight_emul.py c4csg 10 > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; return 1; }
  python3 -c "
import json; d=json.load(open('$O/$n.json'))
print('%-16s w1 %.3f  w8 max %.3f  eff %s' % ('$n', d['w1_f2_max_ms'], d['w8_f2_max_ms'], d.get('w8_f2_eff_max')))"
}
run base "" && run live4 "-DRT_CSG_LIVE=4" && run live5 "-DRT_CSG_LIVE=5" && run live8 "-DRT_CSG_LIVE=8" && \
run grp8 "-DRT_CSG_GROUP_MIN=8" && run grp32 "-DRT_CSG_GROUP_MIN=32" && run sceneglob "" RT_SCENE_GLOBAL=1 && \
run ldslev0 "" RT_LDS_LEVELS=0 && run base2 ""
