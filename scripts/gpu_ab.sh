set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
V=build_variants
timeout -k 10 300 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
timeout -k 10 300 python scripts/ab.py --config c3 --rounds 5 $V/librtamd_prev.so $V/librtamd_base.so $V/librtamd_lf0.so $V/librtamd_lf5.so > gpurun_out/ab.log 2>&1 && \
timeout -k 10 300 python scripts/ab.py --config c4 --rounds 3 $V/librtamd_prev.so $V/librtamd_base.so $V/librtamd_lf0.so $V/librtamd_lf5.so > gpurun_out/ab_c4.log 2>&1 && \
timeout -k 10 300 python scripts/ab.py --config canned --rounds 3 $V/librtamd_prev.so $V/librtamd_base.so > gpurun_out/ab_canned.log 2>&1 && \
timeout -k 10 300 python scripts/ab.py --config c3 --rounds 1 $V/librtamd_phase.so > gpurun_out/phase_c3.log 2>&1
