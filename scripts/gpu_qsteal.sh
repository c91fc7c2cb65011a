# Queue-drain A/B: GPU parity, then strong-scaling rehearsal (incl. a
# one-tile-row share) for RT_QSTEAL variants of the specialised kernel.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/qs
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/qs/pytest.log 2>&1 || { echo "parity failed"; tail -30 gpurun_out/qs/pytest.log; exit 1; }
tail -1 gpurun_out/qs/pytest.log
for f in "" "-DRT_QSTEAL=0" "-DRT_QSTEAL=3" "-DRT_QSTEAL=7"; do
  if [ -n "$f" ]; then export RT_SPEC_EXTRA_FLAGS="$f"; else unset RT_SPEC_EXTRA_FLAGS; fi
  for c in c3 c2; do
    STRONG_WORLDS=1,2,4,8,270 timeout -k 10 300 python3 scripts/strong_emul.py $c > "gpurun_out/qs/$c$f.json" 2> "gpurun_out/qs/$c$f.err" || { echo "strong $c $f failed"; tail -5 "gpurun_out/qs/$c$f.err"; exit 1; }
    echo "[$f] $(cat "gpurun_out/qs/$c$f.json")"
  done
done
