# Frame-stack placement A/B on C3: wall time and calibrated HBM traffic per
# launch for RT_LDS_FULL (levels whose non-core frame fields live in LDS) values.
# usage: bash scripts/gpu_traffic_ab.sh "0 1 2"
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/traffic_ab
mkdir -p $O
timeout -k 10 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/cal_f -o cal_f --output-format csv -- ./build_variants/pmc_calib > /dev/null 2>&1 && \
timeout -k 10 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/cal_w -o cal_w --output-format csv -- ./build_variants/pmc_calib > /dev/null 2>&1 || { echo "calibration failed"; exit 1; }
for v in ${1:-0 1 2}; do
  export RT_LDS_FULL=$v RT_DEBUG_LAUNCH=1
  B="python3 bench.py --config c3 --steps 10 --warmup 2 --cpu-baseline off --companion off"
  timeout -k 10 200 $B > $O/b$v.json 2> $O/b$v.err || { echo "bench $v failed"; tail -3 $O/b$v.err; exit 1; }
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/f$v -o f --output-format csv -- $B > /dev/null 2>&1 && \
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/w$v -o w --output-format csv -- $B > /dev/null 2>&1 || { echo "pmc $v failed"; exit 1; }
  python3 scripts/pmc_traffic.py "$O/[fw]$v/*counter_collection.csv" $O/traffic$v.json "$O/cal_*/*counter_collection.csv" > /dev/null || exit 1
  python3 - <<PY
import json
b = json.load(open("$O/b$v.json")); t = json.load(open("$O/traffic$v.json"))
print("RT_LDS_FULL=$v", b["ms_per_step"], "ms", "read %.3f GB write %.3f GB" % (t["fetch_bytes"] / 1e9, t["write_bytes"] / 1e9))
PY
  grep "\[launch\]" $O/b$v.err | head -1
done
