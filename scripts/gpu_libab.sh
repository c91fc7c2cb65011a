# Whole-frame A/B of the committed library against build_variants/librtamd_old.so
# (and spec flags), with the launch plan printed (RT_DEBUG_LAUNCH).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/libab
mkdir -p $O
run() {  # name lib flags config
  if [ -n "$3" ]; then export RT_SPEC_EXTRA_FLAGS="$3"; else unset RT_SPEC_EXTRA_FLAGS; fi
  RT_AMD_LIB=$2 RT_DEBUG_LAUNCH=1 timeout -k 10 200 python3 bench.py --config $4 --steps 10 --warmup 2 --cpu-baseline off > $O/$1-$4.json 2> $O/$1-$4.err || { echo "bench $1 $4 failed"; tail -5 $O/$1-$4.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/$1-$4.json')); print('$1 $4', d['ms_per_step'], 'ms')"
  grep -m1 "\[launch\]" $O/$1-$4.err || true
}
for c in c4 c3 c4csg; do
  run old build_variants/librtamd_old.so "" $c && \
  run new go-raytracer_amd/csrc/librtamd.so "" $c && \
  run steal7 go-raytracer_amd/csrc/librtamd.so "-DRT_QSTEAL=7" $c || exit 1
done
