# Strong-scaling rehearsal (scripts/strong_emul.py) for variants on one box:
# bash scripts/gpu_strong_ab.sh "<cfgs>" "<variant>" ...   (variant as scripts/gpu_r3_ab.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/strong_ab}
mkdir -p $O
CFGS=$1; shift
for c in $CFGS; do
  for f in "$@"; do
    tag=$(echo "$f" | tr -c 'A-Za-z0-9_=' '_')
    envs=""; flags="$f"
    case "$f" in *"|"*) envs="${f%%|*}"; flags="${f#*|}";; esac
    [ "$flags" = "-" ] && flags=""
    [ "$envs" = "-" ] && envs=""
    if [ -n "$flags" ]; then export RT_SPEC_EXTRA_FLAGS="$flags"; else unset RT_SPEC_EXTRA_FLAGS; fi
    env $envs STRONG_WORLDS=${STRONG_WORLDS:-1,8} timeout -k 10 300 python3 scripts/strong_emul.py $c 10 > $O/$c-$tag.json 2> $O/$c-$tag.err || { tail -5 $O/$c-$tag.err; exit 1; }
    echo "$c [$f] $(cat $O/$c-$tag.json)"
  done
done
