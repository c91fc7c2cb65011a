# Round 5: device-wide sharing knobs, third sweep.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_gshard}
mkdir -p $O
run() {  # name share extra-defines F
  RT_SPEC_EXTRA_FLAGS="$3" INFLIGHT_SHARE=$2 INFLIGHT_F=$4 INFLIGHT_WORLDS=1,8 timeout -k 10 300 python3 scripts/inflight_emul.py c4csg 8 > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; return 1; }
  python3 -c "
import json; d=json.load(open('$O/$1.json')); F=$4
print('%-28s w1 %.3f  w8 max %.3f  eff %s' % ('$1', d['w1_f%d_max_ms' % F], d['w8_f%d_max_ms' % F], d.get('w8_f%d_eff_max' % F)))"
}
run base_f2 0 "" 2 && \
run sh8_p15 2 "" 2 && run sh1_p15 2 "-DRT_GS_SHARDS=1" 2 && \
run sh8_p7 2 "-DRT_GS_POLL=7" 2 && run sh8_p3 2 "-DRT_GS_POLL=3" 2 && \
run sh8_h32 2 "-DRT_GS_HELPERS=32" 2 && run sh8_h64_p7 2 "-DRT_GS_HELPERS=64 -DRT_GS_POLL=7" 2 && \
run sh8_p15_f1 2 "" 1 && run sh8_p15_b 2 "" 2
