# Framebuffer store instructions with and without batched pixel stores (C3):
# SQ_INSTS_VMEM_WR per frame launch (the frame stack's stores included).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/pixw
mkdir -p $O
B="python3 bench.py --config ${1:-c3} --steps 2 --warmup 1 --cpu-baseline off --companion off"
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD -d $O/batch -o p --output-format csv -- $B > /dev/null 2>&1 && \
RT_SPEC_EXTRA_FLAGS=-DRT_PIX_BATCH=0 timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD -d $O/nobatch -o p --output-format csv -- $B > /dev/null 2>&1 || exit 1
for v in batch nobatch; do echo "== $v"; python3 scripts/pmc_summary.py "$O/$v/*counter_collection.csv"; done
