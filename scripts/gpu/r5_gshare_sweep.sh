# Round 5: device-wide sharing knobs (hipRTC defines) on c4csg's 8-rank shares.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_gsweep}
mkdir -p $O
run() {  # name share extra-defines F
  RT_SPEC_EXTRA_FLAGS="$3" INFLIGHT_SHARE=$2 INFLIGHT_F=$4 INFLIGHT_WORLDS=1,8 timeout -k 10 300 python3 scripts/inflight_emul.py c4csg 8 > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; return 1; }
  python3 -c "
import json; d=json.load(open('$O/$1.json')); F=$4
print('%-28s w1 %.3f  w8 max %.3f  eff %s' % ('$1', d['w1_f%d_max_ms' % F], d['w8_f%d_max_ms' % F], d.get('w8_f%d_eff_max' % F)))"
}
run base_f1 0 "" 1 && run dev_f1 2 "" 1 && \
run base_f2 0 "" 2 && run dev_f2 2 "" 2 && \
run dev_min2 2 "-DRT_GS_MIN_LEVELS=2" 2 && run dev_min5 2 "-DRT_GS_MIN_LEVELS=5" 2 && \
run dev_h128 2 "-DRT_GS_HELPERS=128" 2 && run dev_h2048 2 "-DRT_GS_HELPERS=2048" 2 && \
run dev_sleep31 2 "-DRT_SHARE_SLEEP=31" 2 && run grp_f2 1 "" 2
