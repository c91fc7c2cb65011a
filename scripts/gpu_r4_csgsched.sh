# c4csg whole frames (two in flight, 30 steps) under each pixel schedule.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4_${1:-csgsched}
mkdir -p $O
for r in 1 2; do for s in auto pairs quads pixel; do
  timeout -k 10 300 python3 bench.py --config c4csg --steps 30 --warmup 3 --schedule $s --cpu-baseline off --companion off > $O/${s}_r$r.json 2> $O/${s}_r$r.err || { tail -5 $O/${s}_r$r.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/${s}_r$r.json')); print('$s round $r', d['ms_per_step'])"
done; done
