# Brute-force search (bench --accel none: no BVH, no culling) on a full-width
# row band of BASELINE config 5 (7680x4320, 100k spheres): bench line,
# rocprofv3 kernel stats, PMC passes (instruction mix, FP64 counts, waits) and
# the diagnostic build's lane-utilisation counters.
# usage: bash scripts/gpu/brute_pmc.sh TAG [ROWS]     (ROWS default 2048:2304: ~10 pixels per lane, so the tail stays short)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-c5band}
ROWS=${2:-2048:2304}
O=gpurun_out/brute_$TAG
mkdir -p $O
export TMPDIR=/tmp
B="python3 bench.py --config c5 --accel none --rows $ROWS --steps 1 --warmup 1 --inflight 1 --cpu-baseline off"
timeout -k 10 300 $B > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ks -o ks --output-format csv -- $B > /dev/null 2>&1 || { echo "ks failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE -d $O/p1 -o p1 --output-format csv -- $B > /dev/null 2>&1 || { echo "p1 failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAIT_INST_ANY -d $O/p2 -o p2 --output-format csv -- $B > /dev/null 2>&1 || { echo "p2 failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32 -d $O/p4 -o p4 --output-format csv -- $B > /dev/null 2>&1 || { echo "p4 failed"; exit 1; }
python3 scripts/pmc_summary.py "$O/p*/*counter_collection.csv" rt_ > $O/summary.txt && cat $O/summary.txt
find $O/ks -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
cat $O/kernel_stats.csv
if [ -f build_variants/librtamd_phase.so ]; then
  RT_AMD_LIB=build_variants/librtamd_phase.so RT_SPEC_EXTRA_FLAGS="-DRT_PHASE_TIMING -DRT_EXACT_DIAG" timeout -k 10 300 $B > $O/phase.json 2> $O/phase.err || { echo "phase failed"; tail -5 $O/phase.err; exit 1; }
  grep -E "phase|exact|bvh" $O/phase.err | tail -4
fi
python3 scripts/pmc_roofline.py "$O/p[12]/*counter_collection.csv" $O/pmc_roofline.json rt_render
