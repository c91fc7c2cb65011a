# Queue-drain A/B (drained flags + stealing vs home head only): GPU parity,
# strong-scaling rehearsal incl. a one-tile-row share, C3/C4 whole frames.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/qf
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py -x -q --timeout 120 --timeout-method thread \
  > $O/pytest.log 2>&1 || { echo "parity failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for f in "" "-DRT_QSTEAL=0" "-DRT_QSTEAL=3"; do
  if [ -n "$f" ]; then export RT_SPEC_EXTRA_FLAGS="$f"; else unset RT_SPEC_EXTRA_FLAGS; fi
  for c in c3 c4 c2; do
    STRONG_WORLDS=1,2,4,8,270 timeout -k 10 300 python3 scripts/strong_emul.py $c > "$O/$c$f.json" 2> "$O/$c$f.err" || { echo "strong $c $f failed"; tail -5 "$O/$c$f.err"; exit 1; }
    echo "[$f] $(cat "$O/$c$f.json")"
  done
done
