# Round 5: C3 shadow-loop variants after the material-term change freed
# registers: the cull hoist (RT_CULL_HOIST) and the joint culled sweep
# (RT_JOINT_CULL) vs the default; interleaved rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_c3_joint_ab}
mkdir -p $O
b() {  # name flags config
  RT_SPEC_EXTRA_FLAGS="$2" timeout -k 10 300 python3 bench.py --config $3 --steps 20 --warmup 3 --cpu-baseline off --companion off > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/$1.json')); print('%-18s %.4f ms/step' % ('$1', d['ms_per_step']))"
}
for r in 1 2 3; do
  b c3_base$r "" c3 && b c3_hoist$r "-DRT_CULL_HOIST=1" c3 && b c3_joint$r "-DRT_JOINT_CULL=1" c3 || exit 1
done
