# Strong-scaling rehearsal on one GPU for variants (RT_SPEC_EXTRA_FLAGS).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/strong
CFGS=$1; shift
[ $# -eq 0 ] && set -- ""
for c in $CFGS; do
  for f in "$@"; do
    if [ -n "$f" ]; then export RT_SPEC_EXTRA_FLAGS="$f"; else unset RT_SPEC_EXTRA_FLAGS; fi
    timeout -k 10 300 python3 scripts/strong_emul.py $c > "gpurun_out/strong/$c$f.json" 2> "gpurun_out/strong/$c$f.err" || { echo "strong $c $f failed"; tail -5 "gpurun_out/strong/$c$f.err"; exit 1; }
    echo "[$f] $(cat "gpurun_out/strong/$c$f.json")"
  done
done
