# Round 6: diagnostic build (phase split, passes, S_DONE lanes) on the given configs.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/r6_diag}
mkdir -p $O
for c in ${CFGS:-c4csg c3}; do
  RT_AMD_LIB=build_variants/librtamd_phase.so RT_SPEC_EXTRA_FLAGS="-DRT_PHASE_TIMING $XFLAGS" timeout -k 10 300 python3 bench.py --config $c --steps 3 --warmup 1 --cpu-baseline off --companion off $BARGS > $O/$c.json 2> $O/$c.err || { tail $O/$c.err; exit 1; }
  echo "== $c"; grep -E "^\[(phase|passes|lanes|waves)\]" $O/$c.err | tail -4
done
