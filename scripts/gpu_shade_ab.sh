# A/B of the TRACE->SHADE switch threshold (RT_SHADE_NUM/RT_SHADE_DEN) in the
# specialised kernel, C3 / C4 / c3cone, interleaved rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/shade_ab
mkdir -p $O
for r in 1 2; do
for c in c3 c4 c3cone; do
  for f in "" "-DRT_SHADE_NUM=1 -DRT_SHADE_DEN=2" "-DRT_SHADE_NUM=5 -DRT_SHADE_DEN=8" "-DRT_SHADE_NUM=7 -DRT_SHADE_DEN=8"; do
    tag=$(echo "$f" | tr -d ' =-' ); [ -z "$tag" ] && tag=default
    if [ -n "$f" ]; then export RT_SPEC_EXTRA_FLAGS="$f"; else unset RT_SPEC_EXTRA_FLAGS; fi
    timeout -k 10 120 python bench.py --config $c --steps 20 --warmup 2 --cpu-baseline off > $O/$c-$tag-$r.json 2> $O/$c-$tag-$r.err || { echo "$c $tag failed"; tail -5 $O/$c-$tag-$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/$c-$tag-$r.json')); print('$r $c $tag', d['roofline']['kernel_ms'], d['config']['kernel'])"
  done
done
done
