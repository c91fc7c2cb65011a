# Round 5: brute-force C5 band rows 2048-2304, variants via hipRTC defines.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_brute_ab}
mkdir -p $O
run() {
  RT_SPEC_EXTRA_FLAGS="$2" timeout -k 10 300 python3 bench.py --config c5 --accel none --rows 2048:2304 --steps 2 --warmup 1 --cpu-baseline off > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; return 1; }
  python3 -c "
import json; d=json.load(open('$O/$1.json')); r=d['roofline']
print('%-14s band ms %.1f  ref-work frac %.4f' % ('$1', d['ms_per_step'], r.get('reference_work_frac')))"
}
run pairs "" && run quads "-DRT_UNI_PAIRS=2" && run pairs_sc16 "-DRT_SHADOW_CHECK=16" && run quads_sc16 "-DRT_UNI_PAIRS=2 -DRT_SHADOW_CHECK=16" && run pairs2 "" && run quads2 "-DRT_UNI_PAIRS=2"
