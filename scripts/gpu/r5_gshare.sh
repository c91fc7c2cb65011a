# Round 5: device-wide work sharing (RT_SHARE_DEVICE) -- parity, then the
# c4csg 8-rank share rehearsal with and without it.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_gshare}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_schedule.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for sh in 0 2; do
  INFLIGHT_SHARE=$sh INFLIGHT_F=${F:-2} INFLIGHT_WORLDS=1,8 timeout -k 10 400 python3 scripts/inflight_emul.py c4csg 8 > $O/inflight_c4csg_share$sh.json 2> $O/inflight_c4csg_share$sh.err || { tail -5 $O/inflight_c4csg_share$sh.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/inflight_c4csg_share$sh.json'))
print('share=$sh', {k: v for k, v in d.items() if k.endswith('_ms') or 'eff' in k})"
done
# diagnostic build: the board's event counts on rank 0's 8-rank share
RT_AMD_LIB=build_variants/librtamd_phase.so RT_SPEC_EXTRA_FLAGS="-DRT_PHASE_TIMING" INFLIGHT_SHARE=2 INFLIGHT_F=1 INFLIGHT_WORLDS=8 INFLIGHT_RANKS=0 \
  timeout -k 10 300 python3 scripts/inflight_emul.py c4csg 2 > $O/diag_share2.json 2> $O/diag_share2.err || { tail -5 $O/diag_share2.err; exit 1; }
grep -E "share|waves|tail" $O/diag_share2.err | tail -4
