#!/bin/bash
# Offline compile of specialised kernel variants (as hipRTC builds them at run
# time) over a matrix of scene shapes: a backend error ("illegal VGPR to SGPR
# copy" and the like) aborts the process inside hipRTC, so catch it here.
# usage: [SPEC_EXTRA="<options>"] scripts/spec_matrix.sh [jobs]
#   -> prints FAIL lines, exit 1 on any failure (SPEC_EXTRA: options added to
#      every variant, e.g. an RT_SPEC_EXTRA_FLAGS candidate)
R=$(cd "$(dirname "$0")/.." && pwd)
J=${1:-6}
cases=()
# brute force (RT_CULL=0), global linear scenes
for km in 1 3 7 15 31; do for nl in 1 2 3 4 8; do for q in false true; do
  cases+=("-DRT_SPEC_KMASK=$km -DRT_SPEC_FEAT=0 -DRT_SPEC_NLIGHTS=$nl -DRT_SPEC_POWBITS=6 -DRT_CULL=0|false false false $q")
done; done; done
# culled global / BVH / CSG flavours, device-wide sharing
for km in 3 15; do for nl in 2 4; do
  cases+=("-DRT_SPEC_KMASK=$km -DRT_SPEC_FEAT=0 -DRT_SPEC_NLIGHTS=$nl -DRT_SPEC_POWBITS=6|false true false true")
  cases+=("-DRT_SPEC_KMASK=$km -DRT_SPEC_FEAT=0 -DRT_SPEC_NLIGHTS=$nl -DRT_SPEC_POWBITS=6 -DRT_SHARE=2|true true false true")
done; done
for nl in 1 2 3; do
  cases+=("-DRT_SPEC_KMASK=39 -DRT_SPEC_FEAT=0 -DRT_SPEC_NLIGHTS=$nl -DRT_SPEC_POWBITS=6 -DRT_SHARE=2|true false true true")
  cases+=("-DRT_SPEC_KMASK=39 -DRT_SPEC_FEAT=0 -DRT_SPEC_NLIGHTS=$nl -DRT_SPEC_POWBITS=6 -DRT_SHARE=2 -DRT_PAIRS=1|true false true false")
done
# small specialised LDS scenes (unrolled object loops), features, both pixel schedules
for nl in 1 3 4 5 8; do for q in false true; do
  cases+=("-DRT_SPEC_KMASK=15 -DRT_SPEC_FEAT=0 -DRT_SPEC_NOBJ=4 -DRT_SPEC_KINDS=1,3,2,0 -DRT_SPEC_NLIGHTS=$nl -DRT_SPEC_POWBITS=6|true false false $q")
done; done
cases+=("-DRT_SPEC_KMASK=15 -DRT_SPEC_FEAT=7 -DRT_SPEC_NOBJ=8 -DRT_SPEC_KINDS=0,0,0,0,1,2,3,0 -DRT_SPEC_NLIGHTS=8 -DRT_SPEC_POWBITS=7|true false false false")
cases+=("-DRT_SPEC_KMASK=31 -DRT_SPEC_FEAT=7 -DRT_SPEC_NLIGHTS=3 -DRT_SPEC_POWBITS=7|true true false true")
cases+=("-DRT_SPEC_KMASK=15 -DRT_SPEC_FEAT=0 -DRT_SPEC_NOBJ=4 -DRT_SPEC_KINDS=1,3,2,0 -DRT_SPEC_NLIGHTS=4 -DRT_SPEC_POWBITS=6 -DRT_SHARE=1|true false false false")
cases+=("-DRT_SPEC_KMASK=15 -DRT_SPEC_FEAT=0 -DRT_SPEC_NOBJ=4 -DRT_SPEC_KINDS=1,3,2,0 -DRT_SPEC_NLIGHTS=4 -DRT_SPEC_POWBITS=6 -DRT_PAIRS=1|true false false false")
run() {
  IFS='|' read -r defs tmpl <<< "$1"
  defs="$defs ${SPEC_EXTRA:-}"
  out=$(bash "$R/scripts/spec_regs.sh" "$defs" $tmpl 2>&1)
  if echo "$out" | grep -q "error"; then echo "FAIL [$tmpl] $defs: $(echo "$out" | grep error | head -1)"; else echo "ok   [$tmpl] $defs"; fi
}
export -f run; export R SPEC_EXTRA
printf '%s\n' "${cases[@]}" | xargs -P "$J" -I{} bash -c 'run "$@"' _ {} > /tmp/spec_matrix.out
grep FAIL /tmp/spec_matrix.out; n=$(grep -c FAIL /tmp/spec_matrix.out); echo "$(grep -c '^ok' /tmp/spec_matrix.out) ok, $n failed"; [ "$n" = 0 ]
