# C3 bench with F = 2, 3, 4 frames in flight (same box).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4_${1:-inflightF}
mkdir -p $O
for r in 1 2; do for f in 2 3 4; do
  timeout -k 10 300 python3 bench.py --config ${2:-c3} --steps 30 --warmup 3 --inflight $f --cpu-baseline off --companion off > $O/f${f}_r$r.json 2> $O/f${f}_r$r.err || { tail -5 $O/f${f}_r$r.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/f${f}_r$r.json')); print('F=$f round $r', d['ms_per_step'], d['config'].get('schedule'))"
done; done
