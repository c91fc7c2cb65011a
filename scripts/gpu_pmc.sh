set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true
B="python3 bench.py --steps 2 --warmup 1 --cpu-baseline off"
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc/p1 -o p1 --output-format csv -- $B > /dev/null 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAIT_INST_ANY -d gpurun_out/pmc/p2 -o p2 --output-format csv -- $B > /dev/null 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/pmc/p3 -o p3 --output-format csv -- $B > /dev/null 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d gpurun_out/pmc/p4 -o p4 --output-format csv -- $B > /dev/null 2>&1
