# Round 5: the device-wide sharing board's knobs (hipRTC defines) on c4csg's
# rank shares (scripts/inflight_emul.py), one named set per GPU call:
#   bash scripts/gpu/r5_gshare_sweeps.sh poll      -> gpurun_out/r5_gshare_poll/
# Sets, in the order they ran (results: profiles/r05/gshare/r5_gsweep*,
# profiles/r05/gshard, profiles/r05/gpoll):
#   sweep1  frames in flight, subtree depth, helper cap, sleep; the LDS board
#   sweep2  helper cap x subtree depth (one ring)
#   sweep3  small helper caps, poll interval, sleep (one ring)
#   sweep4  longer poll intervals (one ring)
#   sweep5  poll interval; pairs / serial pixel schedules (one ring)
#   shard   per-XCD rings (8) vs one ring, poll, helper cap
#   poll    poll interval, helper cap and depth around the sharded best
# A name's defines are relative to the kernel defaults of the commit it ran at.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
SET=${1:?usage: r5_gshare_sweeps.sh sweep1..5|shard|poll}
O=${O:-gpurun_out/r5_gshare_$SET}
W=${WORLDS:-1,4,8}
mkdir -p $O
run() {  # name share extra-defines F
  RT_SPEC_EXTRA_FLAGS="$3" INFLIGHT_SHARE=$2 INFLIGHT_F=$4 INFLIGHT_WORLDS=$W timeout -k 10 300 python3 scripts/inflight_emul.py c4csg 8 > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; return 1; }
  python3 -c "
import json; d=json.load(open('$O/$1.json')); F=$4
print('%-28s' % '$1', '  '.join('w%d max %.3f (eff %s)' % (w, d['w%d_f%d_max_ms' % (w, F)], d.get('w%d_f%d_eff_max' % (w, F))) for w in (1, 2, 4, 8) if 'w%d_f%d_max_ms' % (w, F) in d))"
}
case $SET in
sweep1)
  run base_f1 0 "" 1 && run dev_f1 2 "" 1 && run base_f2 0 "" 2 && run dev_f2 2 "" 2 && \
  run dev_min2 2 "-DRT_GS_MIN_LEVELS=2" 2 && run dev_min5 2 "-DRT_GS_MIN_LEVELS=5" 2 && \
  run dev_h128 2 "-DRT_GS_HELPERS=128" 2 && run dev_h2048 2 "-DRT_GS_HELPERS=2048" 2 && \
  run dev_sleep31 2 "-DRT_SHARE_SLEEP=31" 2 && run grp_f2 1 "" 2 ;;
sweep2)
  run base_f2 0 "" 2 && \
  for h in 16 32 64 128 256; do run h$h 2 "-DRT_GS_HELPERS=$h" 2 || exit 1; done && \
  for h in 64 128; do for m in 4 5; do run h${h}_m$m 2 "-DRT_GS_HELPERS=$h -DRT_GS_MIN_LEVELS=$m" 2 || exit 1; done; done && \
  run h64_f1 2 "-DRT_GS_HELPERS=64" 1 && run h128_f1 2 "-DRT_GS_HELPERS=128" 1 && run base_f1 0 "" 1 ;;
sweep3)
  run base_f2 0 "" 2 && \
  for h in 4 8 16; do run h$h 2 "-DRT_GS_HELPERS=$h" 2 || exit 1; done && \
  run h16_m4 2 "-DRT_GS_HELPERS=16 -DRT_GS_MIN_LEVELS=4" 2 && run h16_m5 2 "-DRT_GS_HELPERS=16 -DRT_GS_MIN_LEVELS=5" 2 && \
  for p in 7 15 1; do run h16_p$p 2 "-DRT_GS_HELPERS=16 -DRT_GS_POLL=$p" 2 || exit 1; done && \
  run h16_s31 2 "-DRT_GS_HELPERS=16 -DRT_SHARE_SLEEP=31" 2 && run h32_p7 2 "-DRT_GS_HELPERS=32 -DRT_GS_POLL=7" 2 ;;
sweep4)
  run base_f2 0 "" 2 && \
  for p in 15 31 63; do run h16_p$p 2 "-DRT_GS_HELPERS=16 -DRT_GS_POLL=$p" 2 || exit 1; done && \
  run h8_p15 2 "-DRT_GS_HELPERS=8 -DRT_GS_POLL=15" 2 && run h32_p31 2 "-DRT_GS_HELPERS=32 -DRT_GS_POLL=31" 2 && \
  run h16_p15_m4 2 "-DRT_GS_HELPERS=16 -DRT_GS_POLL=15 -DRT_GS_MIN_LEVELS=4" 2 && \
  run h16_p31_m4 2 "-DRT_GS_HELPERS=16 -DRT_GS_POLL=31 -DRT_GS_MIN_LEVELS=4" 2 && \
  run h16_p31_f1 2 "-DRT_GS_HELPERS=16 -DRT_GS_POLL=31" 1 && run base_f1 0 "" 1 ;;
sweep5)
  run base_f2 0 "" 2 && \
  for p in 15 7 3; do run h16_p$p 2 "-DRT_GS_HELPERS=16 -DRT_GS_POLL=$p" 2 || exit 1; done && \
  INFLIGHT_SCHED=pairs run h16_p15_pairs 2 "-DRT_GS_HELPERS=16 -DRT_GS_POLL=15" 2 && \
  INFLIGHT_SCHED=pixel run h16_p15_pixel 2 "-DRT_GS_HELPERS=16 -DRT_GS_POLL=15" 2 && \
  INFLIGHT_SCHED=pairs run base_pairs 0 "" 2 ;;
shard)
  run base_f2 0 "" 2 && run sh8_p15 2 "-DRT_GS_POLL=15" 2 && run sh1_p15 2 "-DRT_GS_SHARDS=1 -DRT_GS_POLL=15" 2 && \
  run sh8_p7 2 "-DRT_GS_POLL=7" 2 && run sh8_p3 2 "-DRT_GS_POLL=3" 2 && \
  run sh8_h32 2 "-DRT_GS_HELPERS=32 -DRT_GS_POLL=15" 2 && run sh8_h64_p7 2 "-DRT_GS_HELPERS=64 -DRT_GS_POLL=7" 2 && \
  run sh8_p15_f1 2 "-DRT_GS_POLL=15" 1 && run sh8_p15_b 2 "-DRT_GS_POLL=15" 2 ;;
poll)
  run p3 2 "-DRT_GS_POLL=3" 2 && run p1 2 "-DRT_GS_POLL=1" 2 && run p0 2 "-DRT_GS_POLL=0" 2 && \
  run p3_h8 2 "-DRT_GS_POLL=3 -DRT_GS_HELPERS=8" 2 && run p3_h32 2 "-DRT_GS_POLL=3 -DRT_GS_HELPERS=32" 2 && \
  run p3_l2 2 "-DRT_GS_POLL=3 -DRT_GS_MIN_LEVELS=2" 2 && run p3_l4 2 "-DRT_GS_POLL=3 -DRT_GS_MIN_LEVELS=4" 2 && \
  run p3_b 2 "-DRT_GS_POLL=3" 2 && run p1_b 2 "-DRT_GS_POLL=1" 2 ;;
*) echo "unknown set $SET"; exit 2 ;;
esac
