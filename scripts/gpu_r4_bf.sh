# Brute-force C5 (scale + translation sphere runs): parity tests, then the
# full-width band timing (rows 2048-2304, bench --accel none) and, if asked,
# PC sampling of C3.  usage: bash scripts/gpu_r4_bf.sh [TAG] [pcs]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-bf}
O=gpurun_out/r4_$TAG
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread -k "brute or axis or synthetic or streamed" > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --config c5 --accel none --rows 2048:2304 --steps 1 --warmup 1 --inflight 1 --cpu-baseline off > $O/band.json 2> $O/band.err || { tail -5 $O/band.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/band.json')); print('c5 bf band', d['roofline']['kernel_ms'], 'ms frac', d['roofline']['frac'])"
if [ "$2" = pcs ]; then bash scripts/gpu_pcsample.sh c3 host_trap; fi
