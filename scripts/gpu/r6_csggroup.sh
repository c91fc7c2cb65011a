# Round 6: c4csg with CSG leaf groups of at most G leaves (RT_CSG_GROUP_LEAVES,
# host-side grouping), interleaved rounds.
# (the RT_CSG_GROUP_LEAVES knob was removed after this measurement: profiles/r06/csg_groups/)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/r6_csggroup}
mkdir -p $O
for r in 1 2; do
  for g in ${GS:-8 4 6}; do
    n=g${g}_r$r
    RT_CSG_GROUP_LEAVES=$g timeout -k 10 300 python3 bench.py --config c4csg --steps 20 --warmup 3 --cpu-baseline off --companion off > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/$n.json')); print('%-8s %.4f ms/step' % ('$n', d['ms_per_step']))"
  done
done
