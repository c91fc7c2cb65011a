# Round 5: the wave index through readfirstlane (an SGPR, RT_WAVE_SGPR=1,
# default) vs the plain VGPR form (0); interleaved rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_wave_ab}
mkdir -p $O
b() {  # name flags config
  RT_SPEC_EXTRA_FLAGS="$2" timeout -k 10 300 python3 bench.py --config $3 --steps 20 --warmup 3 --cpu-baseline off --companion off > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/$1.json')); print('%-18s %.4f ms/step' % ('$1', d['ms_per_step']))"
}
for r in 1 2 3; do
  b c3_w0_$r "-DRT_WAVE_SGPR=0" c3 && b c3_w1_$r "-DRT_WAVE_SGPR=1" c3 && \
  b c2_w0_$r "-DRT_WAVE_SGPR=0" c2 && b c2_w1_$r "-DRT_WAVE_SGPR=1" c2 || exit 1
done
for r in 1 2; do
  b c3cone_w0_$r "-DRT_WAVE_SGPR=0" c3cone && b c3cone_w1_$r "-DRT_WAVE_SGPR=1" c3cone && \
  b c4_w0_$r "-DRT_WAVE_SGPR=0" c4 && b c4_w1_$r "-DRT_WAVE_SGPR=1" c4 && \
  b csg_w0_$r "-DRT_WAVE_SGPR=0" c4csg && b csg_w1_$r "-DRT_WAVE_SGPR=1" c4csg || exit 1
done
