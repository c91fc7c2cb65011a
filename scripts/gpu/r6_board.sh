# Round 6: the device board with explicit acquire points -- the schedule suite
# (incl. the board stress test against the oracle), then the c4csg 8-rank share
# rehearsal (two frames in flight, the default sharing).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/r6_board}
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_schedule.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for rep in 1 2; do
  INFLIGHT_F=2 INFLIGHT_WORLDS=1,8 timeout -k 10 400 python3 scripts/inflight_emul.py c4csg 20 > $O/inflight_c4csg_$rep.json 2> $O/inflight_c4csg_$rep.err || { tail -5 $O/inflight_c4csg_$rep.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/inflight_c4csg_$rep.json'))
print('rep $rep', {k: v for k, v in d.items() if k.endswith('_ms') or 'eff' in k})"
done
