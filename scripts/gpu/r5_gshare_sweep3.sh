# Round 5: device-wide sharing knobs, third sweep.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_gsweep3}
mkdir -p $O
run() {  # name share extra-defines F
  RT_SPEC_EXTRA_FLAGS="$3" INFLIGHT_SHARE=$2 INFLIGHT_F=$4 INFLIGHT_WORLDS=1,8 timeout -k 10 300 python3 scripts/inflight_emul.py c4csg 8 > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; return 1; }
  python3 -c "
import json; d=json.load(open('$O/$1.json')); F=$4
print('%-28s w1 %.3f  w8 max %.3f  eff %s' % ('$1', d['w1_f%d_max_ms' % F], d['w8_f%d_max_ms' % F], d.get('w8_f%d_eff_max' % F)))"
}
run base_f2 0 "" 2 && \
run h4 2 "-DRT_GS_HELPERS=4" 2 && run h8 2 "-DRT_GS_HELPERS=8" 2 && run h16 2 "-DRT_GS_HELPERS=16" 2 && \
run h16_m4 2 "-DRT_GS_HELPERS=16 -DRT_GS_MIN_LEVELS=4" 2 && run h16_m5 2 "-DRT_GS_HELPERS=16 -DRT_GS_MIN_LEVELS=5" 2 && \
run h16_p7 2 "-DRT_GS_HELPERS=16 -DRT_GS_POLL=7" 2 && run h16_p15 2 "-DRT_GS_HELPERS=16 -DRT_GS_POLL=15" 2 && \
run h16_p1 2 "-DRT_GS_HELPERS=16 -DRT_GS_POLL=1" 2 && run h16_s31 2 "-DRT_GS_HELPERS=16 -DRT_SHARE_SLEEP=31" 2 && \
run h32_p7 2 "-DRT_GS_HELPERS=32 -DRT_GS_POLL=7" 2
