# A/B of variants on whole frames: bash scripts/gpu_r3_ab.sh "<cfgs>" "<variant>" ...
# A variant is "ENV=v ENV2=w|<spec flags>" (env for the host library, flags
# for the specialised kernel, RT_SPEC_EXTRA_FLAGS); "-" = defaults.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/r3ab}
ROUNDS=${ROUNDS:-2}
mkdir -p $O
CFGS=$1; shift
for round in $(seq 1 $ROUNDS); do
for c in $CFGS; do
  for f in "$@"; do
    tag=$(echo "$f" | tr -c 'A-Za-z0-9_=' '_')
    envs=""; flags="$f"
    case "$f" in *"|"*) envs="${f%%|*}"; flags="${f#*|}";; esac
    [ "$flags" = "-" ] && flags=""
    [ "$envs" = "-" ] && envs=""
    steps=20; [ $c = c4csg ] && steps=6; [ $c = c5 ] && steps=3
    if [ -n "$flags" ]; then export RT_SPEC_EXTRA_FLAGS="$flags"; else unset RT_SPEC_EXTRA_FLAGS; fi
    env $envs timeout -k 10 300 python bench.py --config $c --steps $steps --warmup 2 --cpu-baseline off --companion off > $O/$c-$tag-$round.json 2> $O/$c-$tag-$round.err || { tail -5 $O/$c-$tag-$round.err; exit 1; }
    echo "r$round $c [$f] $(python3 -c "import json; d=json.load(open('$O/$c-$tag-$round.json')); print(d['ms_per_step'], d['roofline']['kernel_ms'], d['config'].get('tile_order_ms'))")"
  done
done
done
