# PMC passes (scripts/gpu/pmc.sh) for every BASELINE config the bench quotes:
# profiles/pmc_<cfg>.json (executed FP64 work, issue / lane utilisation) and
# profiles/traffic_<cfg>.json (calibrated HBM bytes) land under gpurun_out/pmc_<cfg>/.
# usage: bash scripts/gpu/pmc_all.sh "c3 c3cone c4 c4csg c5"
set -o pipefail
cd $GRAFT_REPO_ROOT
for c in ${1:-c3 c3cone c4 c4csg c5}; do
  # the kernel the in-flight bench runs, one dispatch at a time: C4 whole
  # frames use pixel pairs; c4csg whole frames run without the device board
  # (RT_SHARE_AUTO turns it on for a single frame in flight, which is how
  # these passes dispatch)
  args=""; [ $c = c4 ] && args="--schedule pairs"; [ $c = c4csg ] && args="--work-sharing off"
  PMC_BENCH_ARGS="$args" bash scripts/gpu/pmc.sh $c > gpurun_out/pmc_$c.log 2>&1 || { echo "pmc $c failed"; tail -5 gpurun_out/pmc_$c.log; exit 1; }
  echo "== $c"; tail -2 gpurun_out/pmc_$c.log
done
