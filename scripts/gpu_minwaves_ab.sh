# A/B of the occupancy target (RT_MIN_WAVES, launch bounds) on a
# 64-row full-width band of brute-force C5, two interleaved rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/minwaves_ab
mkdir -p $O
for r in 1 2; do
  for v in 3 4 5; do
    if [ $v != 3 ]; then export RT_SPEC_EXTRA_FLAGS="-DRT_MIN_WAVES=$v"; else unset RT_SPEC_EXTRA_FLAGS; fi
    timeout -k 10 200 python bench.py --config c5 --accel none --rows 2048:2112 --steps 1 --warmup 1 --cpu-baseline off > $O/c5bf-$v-$r.json 2> $O/c5bf-$v-$r.err || { echo "$v failed"; tail -5 $O/c5bf-$v-$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/c5bf-$v-$r.json')); print('$r min_waves=$v', d['roofline']['kernel_ms'], d['roofline']['frac'], d['config']['kernel'])"
  done
done
