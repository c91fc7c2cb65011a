# Deterministic A/B of kernel variants by dynamic instruction counts (one
# rocprofv3 --pmc pass each) plus time: VALU issue slots are what this kernel
# spends (every wave64 VALU instruction, any type, costs an issue slot).
# usage: bash scripts/gpu_valu_ab.sh cfg "ENV=1|flags" ...   (as scripts/gpu_tune.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
CFG=$1; shift
O=gpurun_out/valu_$CFG
mkdir -p $O
export TMPDIR=/tmp
i=0
for fl in "$@"; do
  i=$((i+1))
  envs=""; flags="$fl"
  case "$fl" in *"|"*) envs="${fl%%|*}"; flags="${fl#*|}";; esac
  rm -rf $O/v$i
  env $envs RT_SPEC_EXTRA_FLAGS="$flags" timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_MUL_F64 -d $O/v$i -o v$i --output-format csv -- python3 bench.py --config $CFG --steps 2 --warmup 1 --cpu-baseline off > $O/v$i.json 2> $O/v$i.err || { echo "FAIL v$i"; tail -3 $O/v$i.err; exit 1; }
  python3 - "$O/v$i" "v$i[$fl]" <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "rt_render" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
a = {k: sum(v) / len(v) for k, v in agg.items()}
print(sys.argv[2], " ".join("%s=%.4g" % (k.replace("SQ_", ""), a[k]) for k in sorted(a)))
PY
done
