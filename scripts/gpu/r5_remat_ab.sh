# Round 5: the event counters' LDS addresses formed at each use
# (RT_CNT_REMAT=1) vs hoisted (0, spilled to scratch in C3); kept for the BVH
# and CSG kernels only (the default is now BVH || CSG);
# interleaved rounds over the bench configs.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_remat_ab}
mkdir -p $O
b() {  # name flags config
  RT_SPEC_EXTRA_FLAGS="$2" timeout -k 10 300 python3 bench.py --config $3 --steps 20 --warmup 3 --cpu-baseline off --companion off > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/$1.json')); print('%-18s %.4f ms/step' % ('$1', d['ms_per_step']))"
}
for r in 1 2 3; do
  b c3_r0_$r "-DRT_CNT_REMAT=0" c3 && b c3_r1_$r "-DRT_CNT_REMAT=1" c3 || exit 1
done
for r in 1 2; do
  b c3cone_r0_$r "-DRT_CNT_REMAT=0" c3cone && b c3cone_r1_$r "-DRT_CNT_REMAT=1" c3cone && \
  b c2_r0_$r "-DRT_CNT_REMAT=0" c2 && b c2_r1_$r "-DRT_CNT_REMAT=1" c2 && \
  b c4_r0_$r "-DRT_CNT_REMAT=0" c4 && b c4_r1_$r "-DRT_CNT_REMAT=1" c4 && \
  b csg_r0_$r "-DRT_CNT_REMAT=0" c4csg && b csg_r1_$r "-DRT_CNT_REMAT=1" c4csg || exit 1
done
