# Refresh every judged number at HEAD: round rehearsal (tests, smoke, bench,
# rocprofv3 stats), PMC passes + traffic for C3, the all-config sweep.
set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu_round.sh > gpurun_out/round.log 2>&1 || { tail -30 gpurun_out/round.log; exit 1; }
tail -8 gpurun_out/round.log
bash scripts/gpu_pmc.sh c3 > gpurun_out/pmc.log 2>&1 || { tail -20 gpurun_out/pmc.log; exit 1; }
tail -30 gpurun_out/pmc.log
bash scripts/gpu_sweep.sh || exit 1
for c in c1 c2 canned c3 c4 c4csg c5; do python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['value'], (d.get('cpu_baseline') or {}).get('value'))" gpurun_out/sweep/$c.json $c; done
