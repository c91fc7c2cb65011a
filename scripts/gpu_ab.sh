set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
RT_AMD_LIB=build_variants/librtamd_cp.so timeout -k 10 600 python -m pytest tests -q -m gpu -x > gpurun_out/pytest_gpu_cp.log 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_gpu_cp.log
B=build_variants
V="$B/librtamd_pcull.so $B/librtamd_cp.so go-raytracer_amd/csrc/librtamd.so"
for c in c3 c4 c2; do
timeout -k 10 300 python scripts/ab.py --config $c --rounds 9 $V > gpurun_out/ab_$c.log 2>&1 || exit 1
done
