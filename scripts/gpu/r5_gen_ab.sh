# Round 5: sample-ray divisions through the shared-reciprocal sequence
# (RT_GEN_RCP) vs the hardware division; C3 and C2, interleaved rounds.
# (not kept: the define was removed after this run)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_gen_ab}
mkdir -p $O
b() {  # name flags config
  RT_SPEC_EXTRA_FLAGS="$2" timeout -k 10 300 python3 bench.py --config $3 --steps 20 --warmup 3 --cpu-baseline off --companion off > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/$1.json')); print('%-22s %.4f ms/step' % ('$1', d['ms_per_step']))"
}
for r in 1 2 3; do
  b c3_off$r "-DRT_GEN_RCP=0" c3 && b c3_on$r "-DRT_GEN_RCP=1" c3 && b c2_off$r "-DRT_GEN_RCP=0" c2 && b c2_on$r "-DRT_GEN_RCP=1" c2 || exit 1
done
