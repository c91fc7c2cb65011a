set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
grep -q "pytest rc=0" gpurun_out/pytest_gpu.log || exit 1
B=build_variants
V="$B/librtamd_t_median.so go-raytracer_amd/csrc/librtamd.so"
timeout -k 10 300 python scripts/ab.py --config c4 --rounds 9 $V > gpurun_out/ab_c4.log 2>&1 || exit 1
timeout -k 10 400 python scripts/ab.py --config c5 --rounds 2 $V > gpurun_out/ab_c5.log 2>&1 || exit 1
