# Instruction mix of the C3 kernel (frame dispatches, --inflight 1): two
# rocprofv3 --pmc passes. usage: bash scripts/gpu_r4_mix.sh TAG [CFG] [ENV=...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-mix}; CFG=${2:-c3}
O=gpurun_out/r4_$TAG
mkdir -p $O
B="python3 bench.py --config $CFG --steps 2 --warmup 1 --inflight 1 --cpu-baseline off --companion off"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_BRANCH -d $O/m1 -o m1 --output-format csv -- $B > $O/m1.json 2> $O/m1.err || { echo m1 failed; tail -3 $O/m1.err; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 -d $O/m2 -o m2 --output-format csv -- $B > $O/m2.json 2> $O/m2.err || { echo m2 failed; tail -3 $O/m2.err; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE -d $O/m3 -o m3 --output-format csv -- $B > $O/m3.json 2> $O/m3.err || { echo m3 failed; tail -3 $O/m3.err; exit 1; }
python3 - "$O" <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/m*/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "rt_render" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
# frame dispatches: drop the estimate launch (the smallest)
a = {}
for k, v in agg.items():
    v = sorted(v)[1:] if len(v) > 2 else v
    a[k] = sum(v) / len(v)
print(" ".join("%s=%.4g" % (k.replace("SQ_INSTS_", "").replace("SQ_", ""), a[k]) for k in sorted(a)))
PY
