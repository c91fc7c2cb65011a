set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
timeout -k 10 300 python scripts/ab.py --config c3 --rounds 5 build_variants/librtamd_v1.so build_variants/librtamd_base.so build_variants/librtamd_sh34.so build_variants/librtamd_sh14.so build_variants/librtamd_sh0.so build_variants/librtamd_nocubefast.so > gpurun_out/ab.log 2>&1
