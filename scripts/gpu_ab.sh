set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
grep -q "pytest rc=0" gpurun_out/pytest_gpu.log || exit 1
B=build_variants
V="$B/librtamd_t_base.so go-raytracer_amd/csrc/librtamd.so"
for c in c3 c2 c4; do
timeout -k 10 300 python scripts/ab.py --config $c --rounds 11 $V > gpurun_out/ab_$c.log 2>&1 || exit 1
done
