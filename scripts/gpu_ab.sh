set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B=build_variants
V="go-raytracer_amd/csrc/librtamd.so $B/librtamd_t_near.so"
timeout -k 10 300 python scripts/ab.py --config c4 --rounds 9 $V > gpurun_out/ab_c4.log 2>&1 || exit 1
timeout -k 10 400 python scripts/ab.py --config c5 --rounds 2 $V > gpurun_out/ab_c5.log 2>&1 || exit 1
