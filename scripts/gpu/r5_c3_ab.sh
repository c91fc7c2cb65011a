# Round 5: C3 bench-line A/B of hipRTC define variants (interleaved runs), and
# the c4csg device board's cost on whole frames in flight split into code and
# polling (helpers off + never polling vs the default).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_c3_ab}
mkdir -p $O
b() {  # name defines config [extra bench args]
  n=$1; f=$2; c=$3; shift 3
  RT_SPEC_EXTRA_FLAGS="$f" timeout -k 10 300 python3 bench.py --config $c --steps 20 --warmup 3 --cpu-baseline off --companion off "$@" > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); print('%-16s %.4f ms/step  kernel %.4f' % ('$n', d['ms_per_step'], d['roofline']['kernel_ms']))"
}
# (RT_PLANE_HOIST: +4.6 % on C3, removed after this run -- the define is now a no-op)
for r in 1 2; do b base$r "" c3 && b phoist$r "-DRT_PLANE_HOIST=1" c3 || exit 1; done
for r in 1 2; do
  b csg_off$r "" c4csg --work-sharing off && b csg_dev$r "" c4csg --work-sharing device && \
  b csg_devcode$r "-DRT_GS_HELPERS=0 -DRT_GS_POLL=1048575" c4csg --work-sharing device || exit 1
done
