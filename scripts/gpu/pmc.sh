# PMC passes for the bench kernel (one rocprofv3 run per counter group), plus
# the FETCH_SIZE / WRITE_SIZE calibration for the kernel's access widths.
# usage: bash scripts/gpu/pmc.sh [config]   (default c3)
set -o pipefail
cd $GRAFT_REPO_ROOT
CFG=${1:-c3}
O=gpurun_out/pmc_$CFG
mkdir -p $O
export TMPDIR=/tmp
B="python3 bench.py --config $CFG --steps 2 --warmup 1 --inflight 1 --cpu-baseline off --companion off ${PMC_BENCH_ARGS:-}"
timeout -k 10 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/cal_f -o cal_f --output-format csv -- ./build_variants/pmc_calib > /dev/null 2>&1 && \
timeout -k 10 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/cal_w -o cal_w --output-format csv -- ./build_variants/pmc_calib > /dev/null 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE -d $O/p1 -o p1 --output-format csv -- $B > /dev/null 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAIT_INST_ANY -d $O/p2 -o p2 --output-format csv -- $B > /dev/null 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/p3 -o p3 --output-format csv -- $B > /dev/null 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d $O/p4 -o p4 --output-format csv -- $B > /dev/null 2>&1 && \
python3 scripts/pmc_summary.py "$O/p*/*counter_collection.csv" > $O/summary.txt && \
python3 scripts/pmc_roofline.py "$O/p[12]/*counter_collection.csv" $O/pmc_$CFG.json && \
python3 scripts/pmc_traffic.py "$O/p[34]/*counter_collection.csv" $O/traffic.json "$O/cal_*/*counter_collection.csv" && cat $O/summary.txt $O/traffic.json
