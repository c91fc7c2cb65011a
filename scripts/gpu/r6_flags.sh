# Round 6: compile-flag variants of the specialised kernel (RT_SPEC_EXTRA_FLAGS),
# interleaved rounds on one config.  FLAGSETS: ';'-separated flag sets ("-" = none).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
CFG=${CFG:-c4csg}
O=${O:-gpurun_out/r6_flags_$CFG}
mkdir -p $O
IFS=';' read -ra SETS <<< "${FLAGSETS:--}"
for r in $(seq 1 ${ROUNDS:-2}); do
  i=0
  for f in "${SETS[@]}"; do
    i=$((i+1)); n=v${i}_r$r
    if [ "$f" = "-" ]; then unset RT_SPEC_EXTRA_FLAGS; else export RT_SPEC_EXTRA_FLAGS="$f"; fi
    timeout -k 10 300 python3 bench.py --config $CFG --steps ${STEPS:-20} --warmup 3 --cpu-baseline off --companion off > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/$n.json')); print('%-8s %-40s %.4f ms/step' % ('$n', '$f', d['ms_per_step']))"
  done
done
