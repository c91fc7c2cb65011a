# Headline refresh: C3 PMC passes (executed-work roofline + traffic), default
# bench line, rocprofv3 kernel stats; brute-force C5 band bench + PMC.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_pmc.sh c3 > gpurun_out/pmc_c3.log 2>&1 || { echo "pmc failed"; tail -20 gpurun_out/pmc_c3.log; exit 1; }
tail -2 gpurun_out/pmc_c3.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --cpu-baseline off > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err || { tail gpurun_out/bench_prof.err; exit 1; }
find gpurun_out/prof -name '*kernel_stats.csv' | head -1 | xargs cat
timeout -k 10 300 python3 bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json
bash scripts/gpu_brute_pmc.sh quads > gpurun_out/brute_quads.log 2>&1 || { echo "brute failed"; tail -20 gpurun_out/brute_quads.log; exit 1; }
tail -3 gpurun_out/brute_quads.log
