# Round-3 baseline on a fresh box: default bench line, phase/tail diagnostics
# and the 1-GPU strong-scaling rehearsal of C3 / C4 at HEAD.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/r3base}
mkdir -p $O
timeout -k 10 300 python bench.py --cpu-baseline off > $O/bench_c3.json 2> $O/bench_c3.err || { tail $O/bench_c3.err; exit 1; }
cat $O/bench_c3.json
for c in c3 c4 c4csg; do
  RT_AMD_LIB=build_variants/librtamd_phase.so RT_SPEC_EXTRA_FLAGS="-DRT_PHASE_TIMING" timeout -k 10 200 python bench.py --config $c --steps 3 --warmup 1 --cpu-baseline off > $O/phase_$c.json 2> $O/phase_$c.err || { tail $O/phase_$c.err; exit 1; }
  echo "== $c"; grep -E "phase|waves|tail" $O/phase_$c.err | tail -3
done
for c in c3 c4; do
  timeout -k 10 300 python3 scripts/strong_emul.py $c > $O/strong_$c.json 2> $O/strong_$c.err || { tail -5 $O/strong_$c.err; exit 1; }
  cat $O/strong_$c.json
done
