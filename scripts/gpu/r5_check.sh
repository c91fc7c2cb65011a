# Round 5: the full GPU suite and the bench lines of the kernels a change
# touched (C3, C4, c4csg, the brute-force C5 band).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_check}
mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests -x -q -m gpu --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for c in c3 c4 c4csg; do
  timeout -k 10 300 python3 bench.py --config $c --steps 20 --warmup 3 --cpu-baseline off --companion off > $O/$c.json 2> $O/$c.err || { tail -5 $O/$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$c.json')); print('$c', d['ms_per_step'])"
done
timeout -k 10 300 python3 bench.py --config c5 --accel none --rows 2048:2304 --steps 2 --warmup 1 --cpu-baseline off > $O/band.json 2> $O/band.err || { tail -5 $O/band.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/band.json')); print('band ms', d['ms_per_step'], d['roofline']['reference_work_frac'])"
