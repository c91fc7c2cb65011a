# bench.py over every config (1 GPU), CPU baselines included -> gpurun_out/sweep/
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sweep
for c in c1 c2 canned c3 c4 c4csg c5; do
  steps=10; [ $c = c5 ] && steps=3; [ $c = c4csg ] && steps=3
  timeout -k 10 400 python bench.py --config $c --steps $steps --warmup 1 > gpurun_out/sweep/$c.json 2> gpurun_out/sweep/$c.err || exit 1
done
