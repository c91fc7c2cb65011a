# Round 6: the C3 instruction budget -- dynamic VALU classes (INT32, INT64,
# CVT, F32 add/mul/fma/trans, F64 add/mul/fma/trans, branch, SALU, SMEM, LDS)
# from two rocprofv3 --pmc passes over C3 frames (one at a time, like
# scripts/gpu/pmc.sh), and the phase split of the diagnostic build.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
CFG=${CFG:-c3}
O=${O:-gpurun_out/r6_budget_$CFG}
mkdir -p $O
B="python3 bench.py --config $CFG --steps 2 --warmup 1 --inflight 1 --cpu-baseline off --companion off"
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_BRANCH -d $O/c1 -o c1 --output-format csv -- $B > /dev/null 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SMEM SQ_INSTS_LDS -d $O/c2 -o c2 --output-format csv -- $B > /dev/null 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VSKIPPED SQ_WAVE_CYCLES SQ_INSTS_SENDMSG GRBM_GUI_ACTIVE -d $O/c3 -o c3 --output-format csv -- $B > /dev/null 2>&1 && \
python3 scripts/pmc_summary.py "$O/c*/*counter_collection.csv" > $O/summary.txt && cat $O/summary.txt || exit 1
RT_AMD_LIB=build_variants/librtamd_phase.so RT_SPEC_EXTRA_FLAGS="-DRT_PHASE_TIMING" timeout -k 10 200 python3 bench.py --config $CFG --steps 3 --warmup 1 --cpu-baseline off --companion off > $O/phase.json 2> $O/phase.err || { tail $O/phase.err; exit 1; }
grep -E "phase|waves|passes" $O/phase.err | tail -4
