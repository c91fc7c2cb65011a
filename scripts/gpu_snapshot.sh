# Full measurement snapshot: bench line, rocprof kernel stats, PMC traffic.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/snap
export TMPDIR=/tmp
B="python3 bench.py --steps 3 --warmup 1 --cpu-baseline off"
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/snap/bench.json 2> gpurun_out/snap/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/snap/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --cpu-baseline off > gpurun_out/snap/bench_prof.json 2>gpurun_out/snap/prof.err && \
timeout -k 10 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/snap/pmcT/f -o f --output-format csv -- $B > /dev/null 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/snap/pmcT/w -o w --output-format csv -- $B > /dev/null 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAIT_INST_ANY -d gpurun_out/snap/pmcS/a -o a --output-format csv -- $B > /dev/null 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY -d gpurun_out/snap/pmcS/b -o b --output-format csv -- $B > /dev/null 2>&1
