# Phase / tail diagnostics (RT_PHASE_TIMING build) for spec-flag variants on one box:
# bash scripts/gpu_phase_ab.sh "<cfgs>" "<flags>" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/phase_ab}
mkdir -p $O
CFGS=$1; shift
for c in $CFGS; do
  for f in "$@"; do
    tag=$(echo "$f" | tr -c 'A-Za-z0-9_=' '_')
    [ "$f" = "-" ] && f=""
    RT_AMD_LIB=build_variants/librtamd_phase.so RT_SPEC_EXTRA_FLAGS="-DRT_PHASE_TIMING $f" timeout -k 10 200 python bench.py --config $c --steps 3 --warmup 1 --cpu-baseline off --companion off > $O/$c-$tag.json 2> $O/$c-$tag.err || { tail $O/$c-$tag.err; exit 1; }
    echo "== $c [$f] $(python3 -c "import json; print(json.load(open('$O/$c-$tag.json'))['ms_per_step'])") ms"
    grep -E "phase|waves|tail" $O/$c-$tag.err | tail -3
  done
done
