# C3 with the first levels' full frames (pending refraction ray, first
# child's colour) in LDS (RT_LDS_FULL=n): bench time (same box, two rounds)
# and HBM traffic per frame (FETCH_SIZE / WRITE_SIZE passes, scripts/gpu_pmc.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4_${1:-ldsfull}
mkdir -p $O
for r in 1 2; do for n in 0 1 2 3; do
  RT_LDS_FULL=$n RT_DEBUG_LAUNCH=1 timeout -k 10 300 python3 bench.py --steps 30 --warmup 3 --cpu-baseline off --companion off > $O/n${n}_r$r.json 2> $O/n${n}_r$r.err || { tail -5 $O/n${n}_r$r.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/n${n}_r$r.json')); print('RT_LDS_FULL=$n round $r', d['ms_per_step'])"
  [ $r = 1 ] && grep -m1 "^\[launch\]" $O/n${n}_r$r.err
done; done
for n in 0 2 3; do
  RT_LDS_FULL=$n bash scripts/gpu_pmc.sh c3 > $O/pmc_n$n.log 2>&1 || { tail -5 $O/pmc_n$n.log; exit 1; }
  cp gpurun_out/pmc_c3/traffic.json $O/traffic_n$n.json
  python3 -c "import json; t=json.load(open('$O/traffic_n$n.json')); print('RT_LDS_FULL=$n traffic GB/frame', round(t['traffic_bytes']/1e9, 3) if 'traffic_bytes' in t else t)"
done
