# Round 5: the scheduler's register-pressure trackers (-mllvm
# -amdgpu-use-amdgpu-trackers=1, hipRTC option) on every bench config, and
# combinations on C3; interleaved rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_trackers_ab}
mkdir -p $O
T="-mllvm -amdgpu-use-amdgpu-trackers=1"
b() {  # name flags config [extra bench args]
  n=$1; f=$2; c=$3; shift 3
  RT_SPEC_EXTRA_FLAGS="$f" timeout -k 10 300 python3 bench.py --config $c --steps ${STEPS:-20} --warmup ${WARM:-3} --cpu-baseline off --companion off "$@" > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); print('%-22s %.4f ms/step' % ('$n', d['ms_per_step']))"
}
for r in 1 2; do
  b c3_base$r "" c3 && b c3_trk$r "$T" c3 && b c3_trk_nounc$r "$T -mllvm -amdgpu-disable-unclustered-high-rp-reschedule" c3 && \
  b c3_trk_o2$r "$T -O2" c3 && \
  b c3cone_base$r "" c3cone && b c3cone_trk$r "$T" c3cone && \
  b c2_base$r "" c2 && b c2_trk$r "$T" c2 && \
  b c4_base$r "" c4 && b c4_trk$r "$T" c4 && \
  b csg_base$r "" c4csg && b csg_trk$r "$T" c4csg || exit 1
done
STEPS=3 WARM=1 b c5_base "" c5 && STEPS=3 WARM=1 b c5_trk "$T" c5 && \
STEPS=2 WARM=1 b band_base "" c5 --accel none --rows 2048:2304 && STEPS=2 WARM=1 b band_trk "$T" c5 --accel none --rows 2048:2304
