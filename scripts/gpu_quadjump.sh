# Parity + schedule A/B after a kernel change: GPU parity tests, then C3/C2/C4
# bench with the automatic schedule and with pixel quads forced (RT_PIXEL_QUADS=1).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/qj
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/qj/pytest.log 2>&1 || { echo "parity failed"; tail -30 gpurun_out/qj/pytest.log; exit 1; }
tail -2 gpurun_out/qj/pytest.log
for c in c3 c2 c4csg; do
  for q in auto 1 0; do
    if [ $q = auto ]; then unset RT_PIXEL_QUADS; else export RT_PIXEL_QUADS=$q; fi
    RT_DEBUG_LAUNCH=1 timeout -k 10 300 python3 bench.py --config $c --steps 20 --warmup 2 --cpu-baseline off \
      > gpurun_out/qj/$c-$q.json 2> gpurun_out/qj/$c-$q.err || { echo "bench $c $q failed"; tail -5 gpurun_out/qj/$c-$q.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/qj/$c-$q.json')); print('$c quads=$q', d['ms_per_step'], 'ms')"
    grep -m1 "\[launch\]" gpurun_out/qj/$c-$q.err || true
  done
done
