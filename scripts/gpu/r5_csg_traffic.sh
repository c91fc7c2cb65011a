# Round 5: where c4csg's HBM traffic comes from -- FETCH_SIZE / WRITE_SIZE of
# the default kernel (3 waves/SIMD, 60 VGPRs spilled) against the 2-wave build
# (RT_MIN_WAVES=2: 256 VGPRs, no spills), board off, one dispatch at a time.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in 3 2; do
  O=gpurun_out/csg_traffic_w$v
  RT_SPEC_EXTRA_FLAGS="-DRT_MIN_WAVES=$v" PMC_BENCH_ARGS="--work-sharing off" bash scripts/gpu/pmc.sh c4csg > gpurun_out/csg_traffic_w$v.log 2>&1 || { tail -5 gpurun_out/csg_traffic_w$v.log; exit 1; }
  rm -rf $O && mv gpurun_out/pmc_c4csg $O
  echo "w$v $(python3 -c "import json; t=json.load(open('$O/traffic.json')); print('read %.2f GB write %.2f GB' % (t['fetch_bytes']/1e9, t['write_bytes']/1e9))")"
done
