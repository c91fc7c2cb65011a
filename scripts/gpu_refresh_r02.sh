# Round-2 measurements: C3 PMC passes (executed-work roofline + traffic),
# c3cone (C3 as BASELINE states it), c4csg sweep lines.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sweep
bash scripts/gpu_pmc.sh c3 > gpurun_out/pmc_c3.log 2>&1 || { echo "pmc failed"; tail -20 gpurun_out/pmc_c3.log; exit 1; }
tail -3 gpurun_out/pmc_c3.log
for c in c3cone c4csg; do
  timeout -k 10 400 python bench.py --config $c --steps 5 --warmup 1 > gpurun_out/sweep/$c.json 2> gpurun_out/sweep/$c.err || { echo "bench $c failed"; tail -5 gpurun_out/sweep/$c.err; exit 1; }
  cat gpurun_out/sweep/$c.json
done
