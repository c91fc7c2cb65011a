# Exact (FP64) object tests left after the FP32 culls, per kind, trace and
# shadow (diagnostic build -DRT_PHASE_TIMING -DRT_EXACT_DIAG), serial frames.
# usage: bash scripts/gpu_r4_exact.sh TAG "CFGS"
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; CFGS=${2:-c3}
O=gpurun_out/r4_$TAG
mkdir -p $O
for c in $CFGS; do
  RT_AMD_LIB=build_variants/librtamd_phasex.so RT_SPEC_EXTRA_FLAGS="-DRT_PHASE_TIMING -DRT_EXACT_DIAG" timeout -k 10 300 python3 bench.py --config $c --steps 2 --warmup 1 --inflight 1 --cpu-baseline off --companion off > $O/exact_$c.json 2> $O/exact_$c.err || { tail -5 $O/exact_$c.err; exit 1; }
  echo "== $c"; grep -E "^\[(exact|passes)\]" $O/exact_$c.err | tail -2
done
