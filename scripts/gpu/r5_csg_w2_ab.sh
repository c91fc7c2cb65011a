# Round 5: c4csg whole frames (two in flight) at 3 waves/SIMD (default, 60
# VGPRs spilled) vs 2 (no spills); interleaved rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_csg_w2_ab}
mkdir -p $O
b() {  # name flags config
  RT_SPEC_EXTRA_FLAGS="$2" timeout -k 10 300 python3 bench.py --config $3 --steps 20 --warmup 3 --cpu-baseline off --companion off > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/$1.json')); print('%-14s %.4f ms/step' % ('$1', d['ms_per_step']))"
}
for r in 1 2; do b csg_w3_$r "" c4csg && b csg_w2_$r "-DRT_MIN_WAVES=2" c4csg || exit 1; done
