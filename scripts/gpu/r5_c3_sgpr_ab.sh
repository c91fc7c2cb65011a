# Round 5: the scalar wave index and rematerialised counter addresses
# (RT_WAVE_SGPR, RT_CNT_REMAT) on the small linear kernels, re-measured after
# the material terms freed C3's registers; interleaved rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_c3_sgpr_ab}
mkdir -p $O
b() {  # name flags config
  RT_SPEC_EXTRA_FLAGS="$2" timeout -k 10 300 python3 bench.py --config $3 --steps 20 --warmup 3 --cpu-baseline off --companion off > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/$1.json')); print('%-16s %.4f ms/step' % ('$1', d['ms_per_step']))"
}
for r in 1 2 3; do
  b c3_base$r "" c3 && b c3_w$r "-DRT_WAVE_SGPR=1" c3 && b c3_wr$r "-DRT_WAVE_SGPR=1 -DRT_CNT_REMAT=1" c3 || exit 1
done
for r in 1 2; do
  b c2_base$r "" c2 && b c2_w$r "-DRT_WAVE_SGPR=1" c2 && b c2_wr$r "-DRT_WAVE_SGPR=1 -DRT_CNT_REMAT=1" c2 || exit 1
done
