# Round 6: brute-force C5 band (bench --accel none, rows 2048:2304) A/B of
# libraries, interleaved rounds; VALU / SALU / FP64 counts of each (one
# rocprofv3 --pmc pass per library); then the brute-force and specialised
# parity tests on the working tree's library.
# usage: LIBS="name=path ..." bash scripts/gpu/r6_bf_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/r6_bf_ab}
mkdir -p $O
LIBS=${LIBS:-"head=build_variants/librtamd_head.so new=go-raytracer_amd/csrc/librtamd.so"}
B="python3 bench.py --config c5 --accel none --rows 2048:2304 --steps ${STEPS:-2} --warmup 1 --inflight 1 --cpu-baseline off --companion off"
for r in $(seq 1 ${ROUNDS:-3}); do
  for nl in $LIBS; do
    n=${nl%%=*}; L=${nl#*=}
    RT_AMD_LIB=$L timeout -k 10 300 $B > $O/${n}_r$r.json 2> $O/${n}_r$r.err || { tail -5 $O/${n}_r$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/${n}_r$r.json')); print('%-10s r$r %.1f ms/step' % ('$n', d['ms_per_step']))"
  done
done
if [ -z "$NO_PMC" ]; then
  for nl in $LIBS; do
    n=${nl%%=*}; L=${nl#*=}
    RT_AMD_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_BRANCH SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_ACTIVE_INST_VALU -d $O/pmc_$n -o p --output-format csv -- $B > /dev/null 2>&1 || { echo "pmc $n failed"; exit 1; }
    echo "== $n"; python3 scripts/pmc_summary.py "$O/pmc_$n/*counter_collection.csv" rt_ | grep -E "INSTS|CYCLES|GRBM"
  done
fi
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "brute or c5 or specialised" --timeout 300 --timeout-method thread > $O/pytest_bf.log 2>&1 || { tail -30 $O/pytest_bf.log; exit 1; }
  tail -1 $O/pytest_bf.log
fi
