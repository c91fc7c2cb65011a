# Generic-kernel occupancy: the round-3 fix tree (8eb0a58)
# at 3 waves/SIMD without / with each of its two fixes, then this tree's generic
# kernels at 3 waves/SIMD: reduced-C4 parity, full GPU suite, generic C3 time.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4_generic
mkdir -p $O
B=build_variants
for sz in "96 64" "192 108"; do
  timeout -k 10 300 python3 scripts/generic_parity.py c4 $sz $B/librtamd_r3f0.so $B/librtamd_r3f1.so $B/librtamd_r3f2.so $B/librtamd_r3f3.so $B/librtamd_g3.so go-raytracer_amd/csrc/librtamd.so > "$O/parity_c4_${sz// /x}.log" 2>&1 || { tail -5 "$O/parity_c4_${sz// /x}.log"; exit 1; }
  cat "$O/parity_c4_${sz// /x}.log" | grep -v amdgpu.ids
done
RT_AMD_LIB=$B/librtamd_g3.so timeout -k 10 900 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_g3.log 2>&1; rc=$?; tail -2 $O/pytest_g3.log; [ $rc = 0 ] || exit $rc
for lib in go-raytracer_amd/csrc/librtamd.so $B/librtamd_g3.so; do
  for c in c3 c4 c2; do
    RT_AMD_LIB=$lib timeout -k 10 200 python3 bench.py --config $c --specialize off --inflight 1 --steps 20 --warmup 2 --cpu-baseline off --companion off > $O/gen_${c}_$(basename $lib .so).json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('$O/gen_${c}_$(basename $lib .so).json')); print('$lib $c generic serial', d['roofline']['kernel_ms'], 'ms')"
  done
done
