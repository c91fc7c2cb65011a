# Tuning sweep of the specialised kernel's compile-time knobs (RT_SPEC_EXTRA_FLAGS),
# interleaved over two passes so that clock drift hits every variant alike.
# usage: bash scripts/gpu_tune.sh "cfg1 cfg2" "flags A" "ENV=1 ENV2=2|flags B" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tune
CFGS=$1; shift
for pass in 1 2; do
  for cfg in $CFGS; do
    st=20; [ $cfg = c5 ] && st=3; [ $cfg = c4csg ] && st=5
    i=0
    for fl in "$@"; do
      i=$((i+1))
      envs=""; flags="$fl"
      case "$fl" in *"|"*) envs="${fl%%|*}"; flags="${fl#*|}";; esac
      env $envs RT_SPEC_EXTRA_FLAGS="$flags" timeout -k 10 200 python bench.py --config $cfg --steps $st --warmup 2 --cpu-baseline off > gpurun_out/tune/${cfg}_v${i}_p${pass}.json 2> gpurun_out/tune/${cfg}_v${i}_p${pass}.err || { echo "FAIL $cfg v$i"; tail -5 gpurun_out/tune/${cfg}_v${i}_p${pass}.err; exit 1; }
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], 'ms', d['ms_per_step'], 'kern', d['roofline']['kernel_ms'] if d.get('roofline') else None)" gpurun_out/tune/${cfg}_v${i}_p${pass}.json $cfg "v$i[$fl]"
    done
  done
done
