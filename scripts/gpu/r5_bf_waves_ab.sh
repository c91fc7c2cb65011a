# Round 5: brute-force kernel occupancy (RT_MIN_WAVES 4 / 5 / 6 waves per SIMD)
# on the C5 band after the spill-reload fixes; interleaved rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_bf_waves_ab}
mkdir -p $O
b() {  # name flags
  RT_SPEC_EXTRA_FLAGS="$2" timeout -k 10 300 python3 bench.py --config c5 --accel none --rows 2048:2304 --steps 2 --warmup 1 --cpu-baseline off > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/$1.json')); print('%-12s band ms %.1f  ref-work frac %.4f' % ('$1', d['ms_per_step'], d['roofline']['reference_work_frac']))"
}
for r in 1 2; do b w5_$r "" && b w4_$r "-DRT_MIN_WAVES=4" && b w6_$r "-DRT_MIN_WAVES=6" && b w8_$r "-DRT_MIN_WAVES=8" || exit 1; done
