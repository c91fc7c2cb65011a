set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-baseline off > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 1
timeout -k 10 300 python bench.py --config c2 --steps 20 --warmup 3 --cpu-baseline off > gpurun_out/bench_c2.json 2>> gpurun_out/bench.err || exit 1
