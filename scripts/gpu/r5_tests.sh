# Round 5: the full GPU suite, then the brute-force band and the default bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_tests}
mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests -x -v -m gpu --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python3 bench.py --config c5 --accel none --rows 2048:2304 --steps 2 --warmup 1 --cpu-baseline off > $O/band.json 2> $O/band.err || { tail -5 $O/band.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/band.json')); print('band ms', d['ms_per_step'], d['roofline']['reference_work_frac'])"
