# Diagnostic build on one rank's share (interleaved tile rows, world W, rank
# 0, serial): phase split, wave-lifetime tail, passes.
# usage: bash scripts/gpu_r4_sharediag.sh TAG "CFGS" W
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; CFGS=$2; W=${3:-8}
O=gpurun_out/r4_$TAG
mkdir -p $O
for c in $CFGS; do
  RT_AMD_LIB=build_variants/librtamd_phase.so RT_SPEC_EXTRA_FLAGS="-DRT_PHASE_TIMING" INFLIGHT_WORLDS=1,$W INFLIGHT_F=1 INFLIGHT_RANKS=0 timeout -k 10 300 python3 scripts/inflight_emul.py $c 3 > $O/diag_$c.json 2> $O/diag_$c.err || { tail -5 $O/diag_$c.err; exit 1; }
  echo "== $c"; grep -E "^\[(phase|tail|waves|passes)\]" $O/diag_$c.err | tail -8; cat $O/diag_$c.json
done
