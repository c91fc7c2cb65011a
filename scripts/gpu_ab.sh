set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -q -m gpu -k "cli" > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
B=build_variants
V="$B/librtamd_t_base.so $B/librtamd_t_lf2.so $B/librtamd_t_lf3.so $B/librtamd_t_sh12.so $B/librtamd_t_sh78.so $B/librtamd_t_w3.so $B/librtamd_t_sdiv.so"
for c in c3 c4 c2; do
timeout -k 10 300 python scripts/ab.py --config $c --rounds 7 $V > gpurun_out/ab_$c.log 2>&1 || exit 1
done
