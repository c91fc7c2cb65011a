# C3 frame time and lane utilisation of whole source trees (earlier commits
# built under build_variants/<name>/) against the working tree, on one box.
# usage: bash scripts/gpu_tree_ab.sh "r2 e48e0ef ." [rounds]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/tree_ab
mkdir -p $O
for r in $(seq 1 ${2:-2}); do
  for t in $1; do
    d=$([ "$t" = "." ] && echo . || echo build_variants/$t)
    tag=$(echo $t | tr -c 'A-Za-z0-9' '_')
    extra=$(grep -q -- "--companion" $d/bench.py && echo "--companion off" || echo "")
    (cd $d && timeout -k 10 200 python3 bench.py --config c3 --steps 20 --warmup 3 --cpu-baseline off $extra) > $O/b_${tag}_${r}.json 2> $O/b_$tag.err || { echo "bench $t failed"; tail -3 $O/b_$tag.err; exit 1; }
    echo "round $r $t $(python3 -c "import json;d=json.load(open('$O/b_${tag}_${r}.json'));print(d['ms_per_step'], d['roofline']['kernel_ms'])")"
  done
done
for t in $1; do
  d=$([ "$t" = "." ] && echo . || echo build_variants/$t)
  tag=$(echo $t | tr -c 'A-Za-z0-9' '_')
  extra=$(grep -q -- "--companion" $d/bench.py && echo "--companion off" || echo "")
  (cd $d && timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE SQ_WAVE_CYCLES -d $GRAFT_REPO_ROOT/$O/p_$tag -o p --output-format csv -- python3 bench.py --config c3 --steps 2 --warmup 1 --cpu-baseline off $extra > /dev/null 2>&1) || { echo "pmc $t failed"; exit 1; }
  python3 scripts/pmc_summary.py "$O/p_$tag/*counter_collection.csv" > $O/s_$tag.txt && echo "== $t" && cat $O/s_$tag.txt
done
