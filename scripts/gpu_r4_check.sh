# GPU suite + smoke + the default bench line (with its render_api leg).
# usage: bash scripts/gpu_r4_check.sh [TAG] [pytest -k expr]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4_${1:-check}
mkdir -p $O
K=()
[ -n "$2" ] && K=(-k "$2")
timeout -k 10 900 python3 -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread "${K[@]}" > $O/pytest_gpu.log 2>&1; rc=$?; tail -2 $O/pytest_gpu.log; [ $rc = 0 ] || { grep -E "FAILED|Error|assert" $O/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 400 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -5 $O/bench_default.err; exit 1; }
cat $O/bench_default.json
