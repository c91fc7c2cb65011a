# Pixel pairs: schedule parity tests, then the strong-share rehearsal with pairs forced vs auto.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/pairs}
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_schedule.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc = 0 ] || exit $rc
for c in c3 c4; do
  for v in 0 1; do
    RT_PIXEL_PAIRS=$v INFLIGHT_F=${FS:-1,2} INFLIGHT_WORLDS=${WORLDS:-1,2,4,8} timeout -k 10 300 python3 scripts/inflight_emul.py $c 20 > $O/inflight_${c}_p$v.json 2> $O/inflight_${c}_p$v.err || { tail -5 $O/inflight_${c}_p$v.err; exit 1; }
    echo "$c pairs=$v"; grep -v -e Warn -e amdgpu.ids $O/inflight_${c}_p$v.err
  done
done
