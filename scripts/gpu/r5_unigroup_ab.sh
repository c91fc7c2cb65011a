# Round 5 (grouping not kept and removed; quads kept): brute-force uniform-scale
# runs tested a load group at a time (one
# wave branch per group's real roots, RT_UNI_GROUP=1) vs one branch per sphere
# (0); brute-force parity tests first, then the C5 band, interleaved rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_unigroup_ab}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_synthetic_goldens.py -x -q -m gpu -k "brute or axis or c5" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
b() {  # name flags
  RT_SPEC_EXTRA_FLAGS="$2" timeout -k 10 300 python3 bench.py --config c5 --accel none --rows 2048:2304 --steps 2 --warmup 1 --cpu-baseline off > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/$1.json')); print('%-12s band ms %.1f  ref-work frac %.4f' % ('$1', d['ms_per_step'], d['roofline']['reference_work_frac']))"
}
for r in 1 2; do b old_$r "-DRT_UNI_GROUP=0 -DRT_UNI_PAIRS=1" && b q_$r "-DRT_UNI_GROUP=0" && b qg_$r "" || exit 1; done
