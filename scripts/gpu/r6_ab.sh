# Round 6: A/B of the working tree's library against build_variants/librtamd_head.so
# (the last commit), interleaved bench runs; the VALU / SALU counts of both on
# C3 frames (one rocprofv3 --pmc pass each); then (unless NO_TESTS) the full
# GPU suite on the working tree.
# Knobs: C3_ROUNDS (3), ROUNDS (2), CFGS ("c3cone c2 c4csg"), NO_TESTS, NO_PMC.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/r6_ab}
mkdir -p $O
b() {  # name lib config
  RT_AMD_LIB=$2 timeout -k 10 300 python3 bench.py --config $3 --steps 20 --warmup 3 --cpu-baseline off --companion off > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/$1.json')); print('%-18s %.4f ms/step' % ('$1', d['ms_per_step']))"
}
H=build_variants/librtamd_head.so
N=go-raytracer_amd/csrc/librtamd.so
for r in $(seq 1 ${C3_ROUNDS:-3}); do b c3_head$r $H c3 && b c3_new$r $N c3 || exit 1; done
for r in $(seq 1 ${ROUNDS:-2}); do
  for c in ${CFGS:-c3cone c2 c4csg}; do b ${c}_head$r $H $c && b ${c}_new$r $N $c || exit 1; done
done
if [ -z "$NO_PMC" ]; then
  for v in head new; do
    L=$H; [ $v = new ] && L=$N
    RT_AMD_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU_INT32 SQ_INSTS_BRANCH -d $O/pmc_$v -o p --output-format csv -- python3 bench.py --config ${PMC_CFG:-c3} --steps 2 --warmup 1 --inflight 1 --cpu-baseline off --companion off > /dev/null 2>&1 || exit 1
    echo "== $v"; python3 scripts/pmc_summary.py "$O/pmc_$v/*counter_collection.csv" | grep -E "INSTS|CYCLES"
  done
fi
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 1000 python3 -u -m pytest tests -x -q -m gpu --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
  tail -1 $O/pytest_gpu.log
fi
