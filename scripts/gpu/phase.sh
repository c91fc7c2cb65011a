# Phase split of the (specialised) kernel: diagnostic build with RT_PHASE_TIMING.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
CFG=${1:-c3}; shift
RT_AMD_LIB=build_variants/librtamd_phase.so RT_SPEC_EXTRA_FLAGS="-DRT_PHASE_TIMING $*" timeout -k 10 200 python bench.py --config $CFG --steps 3 --warmup 1 --cpu-baseline off > gpurun_out/phase_$CFG.json 2> gpurun_out/phase_$CFG.err || { tail gpurun_out/phase_$CFG.err; exit 1; }
grep -E "phase|waves|tail" gpurun_out/phase_$CFG.err | tail -3
