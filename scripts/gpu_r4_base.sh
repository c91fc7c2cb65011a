# Round-4 baseline on a fresh box: C3 serial and in-flight bench lines, and the
# diagnostic build's phase split + exact-test counts (build_variants/librtamd_phase.so,
# built on the CPU with -DRT_PHASE_TIMING -DRT_EXACT_DIAG).
# usage: bash scripts/gpu_r4_base.sh [TAG] [CFGS]
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-base}
CFGS=${2:-c3}
O=gpurun_out/r4_$TAG
mkdir -p $O
export TMPDIR=/tmp
for c in $CFGS; do
  timeout -k 10 200 python3 bench.py --config $c --steps 20 --warmup 3 --inflight 1 --cpu-baseline off --companion off > $O/serial_$c.json 2> $O/serial_$c.err || { tail -5 $O/serial_$c.err; exit 1; }
  timeout -k 10 200 python3 bench.py --config $c --steps 20 --warmup 3 --cpu-baseline off --companion off > $O/inflight_$c.json 2> $O/inflight_$c.err || { tail -5 $O/inflight_$c.err; exit 1; }
  python3 -c "import json,sys; a=json.load(open('$O/serial_$c.json')); b=json.load(open('$O/inflight_$c.json')); print('$c serial %.4f ms  inflight %.4f ms/step (kernel %.4f)' % (a['roofline']['kernel_ms'], b['ms_per_step'], b['roofline']['kernel_ms']))"
  if [ -f build_variants/librtamd_phase.so ]; then
    RT_AMD_LIB=build_variants/librtamd_phase.so RT_SPEC_EXTRA_FLAGS="-DRT_PHASE_TIMING -DRT_EXACT_DIAG" timeout -k 10 200 python3 bench.py --config $c --steps 3 --warmup 1 --inflight 1 --cpu-baseline off --companion off > $O/phase_$c.json 2> $O/phase_$c.err || { tail -5 $O/phase_$c.err; exit 1; }
    grep -E "phase|exact|waves|bvh" $O/phase_$c.err | tail -4
  fi
done
