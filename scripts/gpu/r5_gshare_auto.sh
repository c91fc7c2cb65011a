# Round 5: RT_SHARE_AUTO (the default) vs off on c4csg: every rank's share at
# 1/2/4/8 ranks, serial and two in flight; parity suite for the schedules.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_gauto}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_schedule.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for sh in 0 auto; do
  INFLIGHT_SHARE=$sh INFLIGHT_F=1,2 timeout -k 10 400 python3 scripts/inflight_emul.py c4csg 8 > $O/inflight_c4csg_$sh.json 2> $O/inflight_c4csg_$sh.err || { tail -5 $O/inflight_c4csg_$sh.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/inflight_c4csg_$sh.json'))
for F in (1, 2):
    print('share=$sh F=%d' % F, ' '.join('w%d %.3f/%s' % (w, d['w%d_f%d_max_ms' % (w, F)], d.get('w%d_f%d_eff_max' % (w, F))) for w in (1, 2, 4, 8)))"
done
