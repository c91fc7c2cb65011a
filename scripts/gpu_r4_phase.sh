# Phase split (diagnostic build: build_variants/librtamd_phase.so with
# -DRT_PHASE_TIMING, specialised kernel with the same flag), serial launches.
# usage: bash scripts/gpu_r4_phase.sh TAG "CFGS" [extra -D flags]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-phase}; CFGS=${2:-c3}; shift 2
O=gpurun_out/r4_$TAG
mkdir -p $O
for c in $CFGS; do
  RT_AMD_LIB=build_variants/librtamd_phase.so RT_SPEC_EXTRA_FLAGS="-DRT_PHASE_TIMING $*" timeout -k 10 300 python3 bench.py --config $c --steps 3 --warmup 1 --inflight 1 --cpu-baseline off --companion off > $O/phase_$c.json 2> $O/phase_$c.err || { tail -5 $O/phase_$c.err; exit 1; }
  echo "== $c"; grep -E "phase|waves|bvh|passes" $O/phase_$c.err | tail -5
done
