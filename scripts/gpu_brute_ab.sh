# Brute-force C5 (480x270) under compile-time variants of the streamed loop.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/brute_ab
i=0
for fl in "$@"; do
  i=$((i+1))
  RT_SPEC_EXTRA_FLAGS="$fl" timeout -k 10 200 python bench.py --config c5 --width 480 --height 270 --accel none --steps 2 --warmup 1 --cpu-baseline off > gpurun_out/brute_ab/v$i.json 2> gpurun_out/brute_ab/v$i.err || { echo "FAIL v$i"; tail -3 gpurun_out/brute_ab/v$i.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['roofline']['frac'])" gpurun_out/brute_ab/v$i.json "v$i[$fl]"
done
